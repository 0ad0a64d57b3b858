"""Lifted-product code sources (host side, offline): finite groups, their GF(2)
group algebra and regular representations, and the three lifted-product
constructions of the reference, used to produce the larger benchmark codes
(BASELINE configs 3 and 5):

* quasi-cyclic lifted product (PK'20)      -- ``python/qldpc/qc_lifted_product_code.py:16-71``
* matrix lifted product over any group     -- ``python/qldpc/matrix_lifted_product_code.py:105-212``
  (group algebra ``:14-63``, regular representations ``:66-103``)
* Cayley-graph lifted product with local systems, its cyclic and Morgenstern
  wrappers                                 -- ``python/qldpc/lifted_product_code.py:264-453``
* groups: ``Zqm`` (``:106-140``), ``GL2``/``PGL2`` (``:47-104``), ``get_psl2``
  (``:205-212``), Morgenstern generators (``:164-203``), random abelian
  generators (``:142-162``), DFS closure (``:214-234``);
  ``random_check_matrix`` (``python/qldpc/random_code.py:4-22``).

The reference does all field arithmetic with galois (absent here).  This module
carries its own small finite fields (``FiniteField``: GF(p^k) on integer codes in
the polynomial basis of the Conway polynomial -- galois' default -- so element
order, ``primitive_element`` and integer conversions mean the same thing).
Group-algebra coefficients are GF(2) only, which is what every caller in the
reference uses.  Parity is pinned by the reference's own known-answer tests
(``tests/test_qc_lifted_product_code.py``, ``tests/test_matrix_lifted_product_code.py``,
``tests/test_lifted_product_code.py``): code lengths, logical counts and group
orders.  Nothing here runs on the GPU.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from collections import deque
from itertools import product
from typing import Dict, Iterable, List, Sequence

import numpy as np
import scipy.sparse as sp

from .codes import QuantumCode
from .hgp import code_from_boundary_maps

__all__ = [
    "Group", "Zqm", "ZProduct", "FiniteField", "GL2", "PGL2", "get_psl2", "morgenstern_generators",
    "random_abelian_generators", "dfs_generators", "GroupAlgebra", "group_algebra_monomial", "group_algebra_zero",
    "RegularRep", "matrix_lifted_product_code", "qc_lifted_product_code", "bivariate_bicycle_code",
    "random_check_matrix", "lifted_product_code", "lifted_product_code_cyclic", "lifted_product_code_pgl2",
    "psl2_lifted_product_code",
]


# --------------------------------------------------------------------------- groups

class Group(ABC):
    """Minimal group interface (reference ``lifted_product_code.py:20-44``):
    ``a @ b`` is the product, ``inv()``, ``identity()``, hashable values."""

    @abstractmethod
    def __matmul__(self, other):
        ...

    @abstractmethod
    def inv(self):
        ...

    @abstractmethod
    def identity(self):
        ...

    def __pow__(self, n: int):
        assert isinstance(n, int) and n >= 0
        r = self.identity()
        for _ in range(n):
            r = r @ self
        return r


class ZProduct(Group):
    """Abelian group Z_{n_1} x ... x Z_{n_k} (mixed moduli; e.g. Z_12 x Z_6 for the
    [[144,12,12]] bivariate-bicycle code)."""
    __slots__ = ("moduli", "data")

    def __init__(self, moduli: Sequence[int], data: Sequence[int]):
        self.moduli = tuple(int(v) for v in moduli)
        d = tuple(int(v) for v in data)
        if len(d) != len(self.moduli) or any(not 0 <= v < q for v, q in zip(d, self.moduli)):
            raise ValueError("element out of range")
        self.data = d

    def _make(self, data):
        return ZProduct(self.moduli, data)

    def __matmul__(self, other):
        assert self.moduli == other.moduli
        return self._make(tuple((a + b) % q for a, b, q in zip(self.data, other.data, self.moduli)))

    def inv(self):
        return self._make(tuple((-a) % q for a, q in zip(self.data, self.moduli)))

    def identity(self):
        return self._make((0,) * len(self.moduli))

    def __hash__(self):
        return hash((self.moduli, self.data))

    def __eq__(self, other):
        return isinstance(other, ZProduct) and self.moduli == other.moduli and self.data == other.data

    def __repr__(self):
        return f"{type(self).__name__}{self.data}"

    @staticmethod
    def elements(moduli: Sequence[int]) -> List["ZProduct"]:
        return [ZProduct(moduli, d) for d in product(*(range(q) for q in moduli))]


class Zqm(ZProduct):
    """Z_q^m (reference ``lifted_product_code.py:106-140``)."""

    def __init__(self, q: int, m: int, data):
        data = np.asarray(data)
        if data.shape != (m,) or not np.issubdtype(data.dtype, np.integer):
            raise ValueError("Zqm data must be m integers")
        super().__init__((q,) * m, data.tolist())
        self.q, self.m = int(q), int(m)

    def _make(self, data):
        return Zqm(self.q, self.m, np.asarray(data, dtype=np.int64))


# Conway polynomials (coefficients low -> high, leading 1 included) for the small
# fields the constructions use; galois builds GF(p^k) on these by default.
_CONWAY = {
    (2, 1): (1, 1), (2, 2): (1, 1, 1), (2, 3): (1, 1, 0, 1), (2, 4): (1, 1, 0, 0, 1),
    (2, 5): (1, 0, 1, 0, 0, 1), (2, 6): (1, 1, 0, 1, 1, 0, 1), (2, 7): (1, 1, 0, 0, 0, 0, 0, 1),
    (2, 8): (1, 0, 1, 1, 1, 0, 0, 0, 1),
    (3, 2): (2, 2, 1), (3, 3): (1, 2, 0, 1), (5, 2): (2, 4, 1), (7, 2): (3, 6, 1),
}


def _factor_prime_power(q: int):
    for p in range(2, q + 1):
        if q % p == 0:
            k, r = 0, q
            while r % p == 0:
                r //= p
                k += 1
            if r != 1:
                raise ValueError(f"{q} is not a prime power")
            return p, k
    raise ValueError(f"{q} is not a prime power")


class FiniteField:
    """GF(q), q = p^k, elements are the integers 0..q-1 (base-p digits = the
    coefficients in the polynomial basis modulo the Conway polynomial, galois'
    integer representation).  Tables make every operation O(1)."""
    _cache: Dict[int, "FiniteField"] = {}

    def __new__(cls, q: int):
        if q in cls._cache:
            return cls._cache[q]
        self = super().__new__(cls)
        self._build(q)
        cls._cache[q] = self
        return self

    def _build(self, q: int):
        p, k = _factor_prime_power(q)
        self.order, self.characteristic, self.degree = q, p, k
        digits = np.array([[(v // p ** j) % p for j in range(k)] for v in range(q)], dtype=np.int64)
        weights = p ** np.arange(k, dtype=np.int64)
        self.add_table = (((digits[:, None, :] + digits[None, :, :]) % p) @ weights).astype(np.int64)
        self.neg = (((-digits) % p) @ weights).astype(np.int64)
        if k == 1:
            self.mul_table = np.outer(np.arange(q), np.arange(q)) % p
        else:
            if (p, k) not in _CONWAY:
                raise NotImplementedError(f"no Conway polynomial tabulated for GF({p}^{k})")
            mod = np.array(_CONWAY[(p, k)], dtype=np.int64)
            mul = np.zeros((q, q), dtype=np.int64)
            for a in range(q):
                for b in range(a, q):
                    prod = np.convolve(digits[a], digits[b]) % p
                    for deg in range(len(prod) - 1, k - 1, -1):  # reduce modulo the monic Conway polynomial
                        c = prod[deg]
                        if c:
                            prod[deg - k:deg + 1] = (prod[deg - k:deg + 1] - c * mod) % p
                    v = int(prod[:k] @ weights)
                    mul[a, b] = mul[b, a] = v
            self.mul_table = mul
        self.inv_table = np.zeros(q, dtype=np.int64)
        for a in range(1, q):
            self.inv_table[a] = int(np.nonzero(self.mul_table[a] == 1)[0][0])
        self.primitive_element = next(g for g in range(2, q) if self._is_primitive(g)) if q > 2 else 1

    def _is_primitive(self, g: int) -> bool:
        seen, x = 0, 1
        for _ in range(self.order - 1):
            x = int(self.mul_table[x, g])
            seen += 1
            if x == 1:
                break
        return seen == self.order - 1

    @property
    def elements(self):
        return range(self.order)

    def add(self, a, b):
        return int(self.add_table[a, b])

    def sub(self, a, b):
        return int(self.add_table[a, self.neg[b]])

    def mul(self, a, b):
        return int(self.mul_table[a, b])

    def inv(self, a):
        if a == 0:
            raise ZeroDivisionError("0 has no inverse")
        return int(self.inv_table[a])


class GL2(Group):
    """GL(2, q) element ``(a, b, c, d)`` = [[a, b], [c, d]] (reference :47-78)."""
    __slots__ = ("field", "data")

    def __init__(self, field: FiniteField, data):
        self.field = field
        a = np.asarray(data, dtype=np.int64).reshape(2, 2)
        self.data = (int(a[0, 0]), int(a[0, 1]), int(a[1, 0]), int(a[1, 1]))

    def _mul_entries(self, other):
        F = self.field
        a, b, c, d = self.data
        e, f, g, h = other.data
        return (F.add(F.mul(a, e), F.mul(b, g)), F.add(F.mul(a, f), F.mul(b, h)),
                F.add(F.mul(c, e), F.mul(d, g)), F.add(F.mul(c, f), F.mul(d, h)))

    def det(self) -> int:
        F = self.field
        a, b, c, d = self.data
        return F.sub(F.mul(a, d), F.mul(b, c))

    def _inv_entries(self):
        F = self.field
        a, b, c, d = self.data
        r = F.inv(self.det())
        return (F.mul(d, r), F.mul(F.neg[b], r), F.mul(F.neg[c], r), F.mul(a, r))

    def __matmul__(self, other):
        return type(self)(self.field, self._mul_entries(other))

    def inv(self):
        return type(self)(self.field, self._inv_entries())

    def identity(self):
        return type(self)(self.field, (1, 0, 0, 1))

    def __hash__(self):
        return hash((self.field.order, self.data))

    def __eq__(self, other):
        return isinstance(other, GL2) and self.field.order == other.field.order and self.data == other.data

    def __repr__(self):
        return f"{type(self).__name__}(GF({self.field.order}), {self.data})"


class PGL2(GL2):
    """PGL(2, q): GL(2, q) modulo scalars, stored as the representative whose first
    nonzero entry of the top row is 1 (reference :80-104)."""

    def __init__(self, field: FiniteField, data, canonicalized: bool = False):
        super().__init__(field, data)
        if not canonicalized:
            a, b, c, d = self.data
            s = field.inv(a if a != 0 else b)
            self.data = tuple(field.mul(v, s) for v in self.data)

    def __matmul__(self, other):
        return PGL2(self.field, self._mul_entries(other))

    def inv(self):
        return PGL2(self.field, self._inv_entries())

    def identity(self):
        return PGL2(self.field, (1, 0, 0, 1), canonicalized=True)


def get_psl2(q: int) -> frozenset:
    """Image of SL(2, q) in PGL(2, q): order q(q^2-1)/gcd(2, q-1)
    (reference :205-212, same O(q^4) enumeration)."""
    F = FiniteField(q)
    out = set()
    for a, b, c, d in product(F.elements, repeat=4):
        if F.sub(F.mul(a, d), F.mul(b, c)) == 1:
            out.add(PGL2(F, (a, b, c, d)))
    return frozenset(out)


def _canonical_order(elements: Iterable[Group]) -> List[Group]:
    """Deterministic element order: identity first, then by value (the reference
    iterates a hash-ordered set, which varies between interpreter runs)."""
    els = list(elements)
    key = (lambda g: g.data)
    els.sort(key=key)
    ident = els[0].identity()
    els.remove(ident)
    return [ident] + els


def morgenstern_generators(l: int, i: int, use_B_generators: bool = False, symmetric: bool = True) -> List[PGL2]:
    """The q + 1 Morgenstern generators of PGL(2, q^i), q = 2^l, i even
    (reference :164-203, following Dinur et al. arXiv:2111.04808)."""
    assert l >= 1
    if i % 2 != 0:
        raise ValueError("The Morgenstern construction works only for PGL(2, q^i) with even i, "
                         "because we need a quaternion algebra")
    q = 2 ** l
    Fq, Fqi = FiniteField(q), FiniteField(q ** i)
    # i_el not in F_q with i_el^2 + i_el in F_q (integer-code comparison, as the reference)
    i_el = next(x for x in Fqi.elements if x >= q and Fqi.add(Fqi.mul(x, x), x) < q)
    eps = Fqi.add(Fqi.mul(i_el, i_el), i_el)
    pairs = [(g, d) for g, d in product(Fq.elements, Fq.elements)
             if Fq.add(Fq.add(Fq.mul(g, g), Fq.mul(g, d)), Fq.mul(Fq.mul(d, d), eps)) == 1]
    assert len(pairs) == q + 1
    x = Fqi.primitive_element
    gens = []
    for g, d in pairs:
        top = Fqi.add(g, Fqi.mul(d, i_el))
        bot = Fqi.mul(x, Fqi.add(Fqi.add(g, d), Fqi.mul(d, i_el)))
        gens.append(PGL2(Fqi, (1, top, bot, 1)))
    if use_B_generators:
        gens = [a @ b for s, a in enumerate(gens) for t, b in enumerate(gens) if s != t and (s < t or symmetric)]
    return gens


def random_abelian_generators(q: int, m: int, k: int, symmetric: bool = False, seed=None) -> List[Zqm]:
    """k random elements of Z_q^m; with ``symmetric`` k/2 of them plus inverses
    (reference :142-162, same numpy draws)."""
    rng = np.random.default_rng(seed)
    symmetrize = bool(symmetric) and q != 2
    if symmetrize:
        if k % 2:
            raise ValueError("Number of generators must be even when the set is symmetrized and q /= 2")
        k //= 2
    rows = rng.integers(low=0, high=q, size=(k, m))
    gens = [Zqm(q, m, rows[j]) for j in range(k)]
    if symmetrize:
        gens = [h for g in gens for h in (g, g.inv())]
    return gens


def dfs_generators(root: Group, generators: Sequence[Group], traverse=None) -> List[Group]:
    """Closure of ``root`` under right multiplication by the generators (the
    group they generate when root is the identity; reference :214-234).  Returned
    in canonical order (identity first)."""
    step = traverse or (lambda a, b: a @ b)
    seen = set()
    todo = deque([root])
    while todo:
        x = todo.pop()
        if x in seen:
            continue
        seen.add(x)
        todo.extend(step(x, g) for g in generators)
    return _canonical_order(seen)


# --------------------------------------------------------------------------- group algebra F2[G]

class GroupAlgebra:
    """Element of F2[G]: the set of group elements with coefficient 1
    (reference ``matrix_lifted_product_code.py:14-63`` restricted to GF(2))."""
    __slots__ = ("support",)

    def __init__(self, support: Iterable[Group] = ()):
        s = set()
        for g in support:  # repeated terms cancel mod 2
            s ^= {g}
        self.support = frozenset(s)

    def __add__(self, other):
        return GroupAlgebra(self.support ^ other.support)

    def __mul__(self, other):
        if isinstance(other, GroupAlgebra):
            return GroupAlgebra(a @ b for a in self.support for b in other.support)
        return self if int(other) % 2 else GroupAlgebra()

    __rmul__ = __mul__

    def antipode(self):
        return GroupAlgebra(g.inv() for g in self.support)

    def terms(self):
        return {g: 1 for g in self.support}

    def __eq__(self, other):
        return isinstance(other, GroupAlgebra) and self.support == other.support

    def __hash__(self):
        return hash(self.support)

    def __repr__(self):
        return f"GroupAlgebra({sorted(map(repr, self.support))})"


def group_algebra_zero(*_):
    return GroupAlgebra()


def group_algebra_monomial(*args):
    """``group_algebra_monomial(element)`` or the reference's
    ``group_algebra_monomial(scale, element)`` with a GF(2) scale."""
    if len(args) == 1:
        return GroupAlgebra([args[0]])
    scale, element = args
    return GroupAlgebra([element]) if int(scale) % 2 else GroupAlgebra()


class RegularRep:
    """Left (h = element @ g) or right (h = g @ element) regular representation of
    a finite group as 0/1 permutation matrices; rows index h, columns index g
    (reference ``matrix_lifted_product_code.py:66-103``)."""

    def __init__(self, group: Sequence[Group], field=None, right_action: bool = False):
        self.group = list(group)
        self.index = {g: t for t, g in enumerate(self.group)}
        self.right_action = bool(right_action)
        self._perm: Dict[Group, np.ndarray] = {}

    def permutation(self, element: Group) -> np.ndarray:
        """perm[col g] = row index of the image of g."""
        p = self._perm.get(element)
        if p is None:
            if self.right_action:
                p = np.array([self.index[g @ element] for g in self.group], dtype=np.int64)
            else:
                p = np.array([self.index[element @ g] for g in self.group], dtype=np.int64)
            self._perm[element] = p
        return p

    def get_rep(self, element: Group) -> np.ndarray:
        n = len(self.group)
        m = np.zeros((n, n), dtype=np.uint8)
        m[self.permutation(element), np.arange(n)] = 1
        return m

    def zero(self) -> np.ndarray:
        n = len(self.group)
        return np.zeros((n, n), dtype=np.uint8)


def _lift_blocks(blocks: Dict[tuple, GroupAlgebra], shape, rep: RegularRep) -> sp.csr_matrix:
    """Binary matrix of a block matrix over F2[G]: block (I, J) is the sum of the
    representation matrices of its terms."""
    N = len(rep.group)
    rows, cols = [], []
    cidx = np.arange(N, dtype=np.int64)
    for (I, J), a in blocks.items():
        for g in a.support:
            rows.append(I * N + rep.permutation(g))
            cols.append(J * N + cidx)
    if rows:
        r, c = np.concatenate(rows), np.concatenate(cols)
    else:
        r = c = np.zeros(0, dtype=np.int64)
    m = sp.coo_matrix((np.ones(r.size, dtype=np.int64), (r, c)), shape=(shape[0] * N, shape[1] * N)).tocsr()
    m.data %= 2
    m.eliminate_zeros()
    return m


def _kron_identity_blocks(A, size: int, left: bool):
    """Nonzero blocks of kron(A, I_size) (left=True) or kron(I_size, A)."""
    a0, a1 = A.shape
    out = {}
    for i in range(a0):
        for j in range(a1):
            if not A[i, j].support:
                continue
            for k in range(size):
                key = (i * size + k, j * size + k) if left else (k * a0 + i, k * a1 + j)
                out[key] = A[i, j]
    shape = (a0 * size, a1 * size)
    return out, shape


def _as_ga_matrix(a) -> np.ndarray:
    a = np.asarray(a, dtype=object)
    if a.ndim != 2:
        raise ValueError("base matrix must be 2-d")
    return a


def matrix_lifted_product_code(group: Sequence[Group], base_matrix_A, base_matrix_B=None, dual_A=None, dual_B=None,
                               check_complex=None, compute_logicals=None) -> QuantumCode:
    """Lift of the tensor product of the complexes A: A1 -> A0 and B: B1 -> B0
    with entries in F2[G] (reference ``matrix_lifted_product_code.py:105-212``).

    B defaults to A* (transpose + antipode).  The A factor acts by the left
    regular representation, the B factor by the right one, so the lifted
    boundary maps compose to zero for any finite group:
    ``partial_2 = [L(A (x) I_B1) ; R(I_A1 (x) B)]``,
    ``partial_1 = [R(I_A0 (x) B) | L(A (x) I_B0)]``."""
    if base_matrix_B is None:
        assert dual_A is None and dual_B is None
    A = _as_ga_matrix(base_matrix_A)

    def dual(m):
        t = m.T
        return np.vectorize(lambda x: x.antipode(), otypes=[object])(t)

    B = dual(A) if base_matrix_B is None else _as_ga_matrix(base_matrix_B)
    if dual_A:
        A = dual(A)
    if dual_B:
        B = dual(B)
    group = list(group)
    left, right = RegularRep(group), RegularRep(group, right_action=True)
    (a0, a1), (b0, b1) = A.shape, B.shape

    top, top_shape = _kron_identity_blocks(A, b1, left=True)        # A (x) I_B1 : A1xB1 -> A0xB1
    bot, bot_shape = _kron_identity_blocks(B, a1, left=False)       # I_A1 (x) B : A1xB1 -> A1xB0
    p2 = sp.vstack([_lift_blocks(top, top_shape, left), _lift_blocks(bot, bot_shape, right)])
    lhs, lhs_shape = _kron_identity_blocks(B, a0, left=False)       # I_A0 (x) B : A0xB1 -> A0xB0
    rhs, rhs_shape = _kron_identity_blocks(A, b0, left=True)        # A (x) I_B0 : A1xB0 -> A0xB0
    p1 = sp.hstack([_lift_blocks(lhs, lhs_shape, right), _lift_blocks(rhs, rhs_shape, left)])
    return code_from_boundary_maps(p2, p1, compute_logicals=bool(compute_logicals),
                                   check_complex=bool(check_complex))


def _poly_terms(entry) -> List[int]:
    """Exponents of a quasi-cyclic entry: an int shift k (x^k), a sequence of
    exponents (sum of monomials), or None / negative for the zero polynomial."""
    if entry is None:
        return []
    if isinstance(entry, (int, np.integer)):
        return [] if entry < 0 else [int(entry)]
    return [int(e) for e in entry]


def qc_lifted_product_code(quasicyclic_check_matrix, l: int, check_complex=None, compute_logicals=None) -> QuantumCode:
    """Quasi-cyclic lifted product of arXiv:2012.04068 (reference
    ``qc_lifted_product_code.py:16-71``): entries of the base matrix live in
    F2[x]/(x^l - 1) and B = A* (x^k -> x^{-k}).  Each monomial x^k lifts to the
    l x l circulant with ones at (j + k mod l, j), i.e. the regular representation
    of Z_l, so this is ``matrix_lifted_product_code`` over Z_l."""
    Zl = ZProduct.elements((l,))
    a = np.asarray(quasicyclic_check_matrix, dtype=object)
    A = np.empty(a.shape, dtype=object)
    for idx in np.ndindex(a.shape):
        A[idx] = GroupAlgebra(Zl[e % l] for e in _poly_terms(a[idx]))
    return matrix_lifted_product_code(Zl, A, check_complex=check_complex, compute_logicals=compute_logicals)


def bivariate_bicycle_code(l: int, m: int, a_terms, b_terms, compute_logicals=None) -> QuantumCode:
    """Bivariate-bicycle code over Z_l x Z_m (Bravyi et al. 2024) as a matrix
    lifted product with 1x1 base matrices [a] and [b]: Hx = [L(a)^T | R(b)^T],
    Hz = [R(b) | L(a)].  ``a_terms``/``b_terms`` are (i, j) exponents of x^i y^j.
    ``bivariate_bicycle_code(12, 6, [(3,0),(0,1),(0,2)], [(0,3),(1,0),(2,0)])`` is
    the [[144,12,12]] code (BASELINE config 3)."""
    els = ZProduct.elements((l, m))
    ga = lambda terms: GroupAlgebra(ZProduct((l, m), (i % l, j % m)) for i, j in terms)
    A = np.empty((1, 1), dtype=object)
    B = np.empty((1, 1), dtype=object)
    A[0, 0], B[0, 0] = ga(a_terms), ga(b_terms)
    return matrix_lifted_product_code(els, A, B, compute_logicals=compute_logicals)


def psl2_lifted_product_code(q: int, rows: int = 3, cols: int = 6, seed: int = 0, compute_logicals=None) -> QuantumCode:
    """Matrix lifted product over PSL(2, q) with a ``rows x cols`` base matrix of
    random monomials and B = A* (the reference's ``test_psl_lift`` shape,
    ``tests/test_matrix_lifted_product_code.py:43-62``).  n = (rows^2 + cols^2)|G|;
    q = 13 gives n = 45 * 1092 = 49,140 (BASELINE config 5)."""
    group = _canonical_order(get_psl2(q))
    rng = np.random.default_rng(seed)
    picks = rng.integers(0, len(group), size=(rows, cols))
    A = np.empty((rows, cols), dtype=object)
    for idx in np.ndindex(A.shape):
        A[idx] = GroupAlgebra([group[int(picks[idx])]])
    return matrix_lifted_product_code(group, A, compute_logicals=compute_logicals)


# --------------------------------------------------------------------------- Cayley-graph lifted product

def random_check_matrix(r: int, n: int, seed=None, full_rank: bool = False) -> np.ndarray:
    """Random r x n GF(2) matrix, rejection-sampled to full rank on request
    (reference ``random_code.py:4-22``, same numpy draws)."""
    from .gf2 import rank
    rng = np.random.default_rng(seed)
    for _ in range(10000):
        h = rng.integers(low=0, high=2, size=(r, n))
        if not full_rank or rank(h) == min(h.shape):
            return h.astype(np.uint8)
    raise RuntimeError("Failed to construct random matrix: Number of retries exceeded")


def lifted_product_code(group: Sequence[Group], generators: Sequence[Group], h1, h2, check_complex=None,
                        compute_logicals=None, double_cover=None, base_graph=None) -> QuantumCode:
    """Lifted product of two Cayley-graph complexes with local systems h1, h2
    (reference ``lifted_product_code.py:264-409``).

    Base graph: generator k is a directed edge 0 -> 1 (double cover, default) or a
    self-loop 0 -> 0.  Every node indexes its incident edges out-edges first, then
    in-edges; h1/h2 columns follow that order.  Cells, each times G:
    qubits E x E (+) (V, h1 rows) x (V, h2 rows); X checks E x (V, h2 rows);
    Z checks (V, h1 rows) x E.  The left factor's group action is from the
    left (e.g. head of e1 contributes ``gen(e1) @ g``), the right factor's from the
    right (in-edges of v2 contribute ``g @ gen(e2)^-1``), as in the reference;
    the cell orders also follow the reference's iteration order."""
    double_cover = True if double_cover is None else double_cover
    h1 = np.asarray(h1) % 2
    h2 = np.asarray(h2) % 2
    if h1.shape[1] != h2.shape[1]:
        raise ValueError("Local code block lengths must match. (For now)")
    group = list(group)
    gidx = {g: t for t, g in enumerate(group)}
    G = len(group)
    if base_graph is None:
        nodes = [0, 1] if double_cover else [0]
        edges = [(0, 1 if double_cover else 0, g) for g in generators]
    else:
        nodes = list(base_graph.nodes)
        edges = [(u, v, d["g"]) for u, v, d in base_graph.edges(data=True)]
    E, V = len(edges), len(nodes)
    vpos = {v: t for t, v in enumerate(nodes)}
    out_idx, in_idx = {}, {}
    for v in nodes:
        outs = [k for k, e in enumerate(edges) if e[0] == v]
        ins = [k for k, e in enumerate(edges) if e[1] == v]
        out_idx[v] = {k: t for t, k in enumerate(outs)}
        in_idx[v] = {k: t + len(outs) for t, k in enumerate(ins)}
        if len(outs) + len(ins) != h1.shape[1]:
            raise ValueError("Local code block length does not match base graph degree")
    r1s, r2s = h1.shape[0], h2.shape[0]
    # group actions as index permutations: left multiplication by gen(e), right by gen(e)^-1
    lmul = [np.array([gidx[e[2] @ g] for g in group], dtype=np.int64) for e in edges]
    rmul_inv = [np.array([gidx[g @ e[2].inv()] for g in group], dtype=np.int64) for e in edges]
    garange = np.arange(G, dtype=np.int64)

    def ee(e1, g, e2):  # qubit E x E
        return (e1 * G + g) * E + e2

    n_ee = E * G * E

    def vv(v1, r1, g, v2, r2):  # qubit (V,h1) x (V,h2)
        return n_ee + ((((v1 * r1s + r1) * G + g) * V + v2) * r2s + r2)

    def xc(e1, v2, r2, g):
        return ((e1 * V + v2) * r2s + r2) * G + g

    def zc(v1, r1, g, e2):
        return ((v1 * r1s + r1) * G + g) * E + e2

    n_q = n_ee + (V * r1s) * (V * r2s) * G
    n_x = E * V * r2s * G
    n_z = V * r1s * G * E
    # X checks: rows of Hx (= columns of partial_2)
    xr, xq = [], []
    for k1, (u1, v1, _) in enumerate(edges):
        hv = h1[:, in_idx[v1][k1]].nonzero()[0]
        hu = h1[:, out_idx[u1][k1]].nonzero()[0]
        for v2 in nodes:
            p2 = vpos[v2]
            for r2 in range(r2s):
                rows = xc(k1, p2, r2, garange)
                for r1 in hv:
                    xr.append(rows); xq.append(vv(vpos[v1], r1, lmul[k1], p2, r2))
                for r1 in hu:
                    xr.append(rows); xq.append(vv(vpos[u1], r1, garange, p2, r2))
                for k2 in out_idx[v2]:
                    if h2[r2, out_idx[v2][k2]]:
                        xr.append(rows); xq.append(ee(k1, garange, k2))
                for k2 in in_idx[v2]:
                    if h2[r2, in_idx[v2][k2]]:
                        xr.append(rows); xq.append(ee(k1, rmul_inv[k2], k2))
    # Z checks: rows of Hz (= partial_1)
    zr, zq = [], []
    for k1, (u1, v1, _) in enumerate(edges):
        hv = h1[:, in_idx[v1][k1]].nonzero()[0]
        hu = h1[:, out_idx[u1][k1]].nonzero()[0]
        for k2 in range(E):
            q = ee(k1, garange, k2)
            for r1 in hv:
                zq.append(q); zr.append(zc(vpos[v1], r1, lmul[k1], k2))
            for r1 in hu:
                zq.append(q); zr.append(zc(vpos[u1], r1, garange, k2))
    for v1 in nodes:
        for r1 in range(r1s):
            for v2 in nodes:
                for r2 in range(r2s):
                    q = vv(vpos[v1], r1, garange, vpos[v2], r2)
                    for k2 in out_idx[v2]:
                        if h2[r2, out_idx[v2][k2]]:
                            zq.append(q); zr.append(zc(vpos[v1], r1, garange, k2))
                    for k2 in in_idx[v2]:
                        if h2[r2, in_idx[v2][k2]]:
                            zq.append(q); zr.append(zc(vpos[v1], r1, rmul_inv[k2], k2))

    def build(r, c, shape):
        r = np.concatenate(r) if r else np.zeros(0, dtype=np.int64)
        c = np.concatenate(c) if c else np.zeros(0, dtype=np.int64)
        m = sp.coo_matrix((np.ones(r.size, dtype=np.int64), (r, c)), shape=shape).tocsr()
        m.data %= 2  # redundant incidences cancel (reference :394-396)
        m.eliminate_zeros()
        return m

    hx = build(xr, xq, (n_x, n_q))
    hz = build(zr, zq, (n_z, n_q))
    return code_from_boundary_maps(hx.T, hz, compute_logicals=bool(compute_logicals),
                                   check_complex=bool(check_complex))


def _lp_wrapper(generators, r, compute_logicals, seed, check_complex, r2=None, double_cover=None) -> QuantumCode:
    """Reference ``_lifted_product_code_wrapper`` (:411-428): group = closure of the
    generators; random local systems seeded with seed+1 / seed+2."""
    assert r > 0
    r2 = r if r2 is None else r2
    compute_logicals = True if compute_logicals is None else compute_logicals
    w = len(generators)
    group = dfs_generators(generators[0].identity(), generators)
    width = w if double_cover else 2 * w
    h1 = random_check_matrix(r, width, seed=None if seed is None else seed + 1)
    h2 = random_check_matrix(r2, width, seed=None if seed is None else seed + 2)
    return lifted_product_code(group, generators, h1, h2, check_complex=check_complex,
                               compute_logicals=compute_logicals, double_cover=double_cover)


def lifted_product_code_cyclic(q, m, w, r, compute_logicals=None, r2=None, seed=None, check_complex=None,
                               double_cover=None) -> QuantumCode:
    """LP code on w random generators of Z_q^m (reference :430-445)."""
    assert q > 0 and m > 0 and w > 0
    double_cover = False if double_cover is None else double_cover
    gens = random_abelian_generators(q, m, w, seed=seed)
    return _lp_wrapper(gens, r, compute_logicals=compute_logicals, r2=r2, seed=seed, check_complex=check_complex,
                       double_cover=double_cover)


def lifted_product_code_pgl2(l, i, r, compute_logicals=None, seed=None, check_complex=None, r2=None,
                             double_cover=None) -> QuantumCode:
    """LP code on the Morgenstern generators of PGL(2, (2^l)^i) (reference :447-453)."""
    gens = morgenstern_generators(l, i)
    return _lp_wrapper(gens, r, compute_logicals=compute_logicals, r2=r2, seed=seed, check_complex=check_complex,
                       double_cover=double_cover)
