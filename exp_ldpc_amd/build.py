"""Build libqdec_hip.so in-tree with hipcc for gfx950.

``python -m exp_ldpc_amd.build`` (also called by ``__graft_entry__.build()``).
The library is built here (hipcc cross-compiles without a GPU) and travels to the
GPU box with the repository snapshot.

Numerics flags: ``-ffp-contract=off`` (no fused multiply-add: every operation is
rounded like the CPU oracle and ldpc's loops), IEEE fp32 division, fp32
denormals kept.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libqdec_hip.so")
SOURCES = ["qdec_abi.cpp", "qdec_osd.cpp", "qdec_gf2.cpp", "qdec_hgp.cpp", "qdec_bp.hip", "qdec_bp_block.hip",
           "qdec_sample.hip", "qdec_osd.hip"]
# device source compiled at run time (hipRTC, per hypergraph-product code): embedded
# into the library as a string literal (build/gen/qdec_hgp_src.inc)
RTC_SOURCES = ["qdec_hgp_kernel.hip"]
HEADERS = [os.path.basename(p) for p in glob.glob(os.path.join(CSRC, "*.h"))] + ["../../include/qdec.h"]
ARCH = os.environ.get("QDEC_OFFLOAD_ARCH", "gfx950")

FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
    "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
    "-Wall", "-Wno-unused-result", "-pthread", f'-DQDEC_ARCH="{ARCH}"',
]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: cannot build libqdec_hip.so")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS + RTC_SOURCES] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


# host-only ASan + UBSan variant (tools/sanitize.sh): every -fsanitize=
# applies to the host compilation only (-Xarch_host), the device code is the
# product's; the runtime comes from the process (LD_PRELOAD of clang's libasan)
SAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
             "-Xarch_host", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g"]
SAN_LINK = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-shared-libsan"]


def build(force: bool = False, verbose: bool = False, stamps: bool = False, defines=(), tag: str = "",
          flags=(), link_flags=()) -> str:
    """Build the library; stamps=True builds the development variant with phase
    timers (libqdec_hip_stamps.so), `defines` + `tag` a development variant
    (libqdec_hip_<tag>.so); variants are loaded with QDEC_LIB=....  Every source
    is compiled to its own object in parallel (objects under build/, git-ignored),
    then linked."""
    from concurrent.futures import ThreadPoolExecutor
    suffix = ("_stamps" if stamps else "") + (f"_{tag}" if tag else "")
    lib = LIB.replace(".so", suffix + ".so")
    if not force and not suffix and not _stale():
        return LIB
    extra = (["-DQDEC_STAMPS"] if stamps else []) + [f"-D{d}" for d in defines] + list(flags)
    objdir = os.path.join(os.path.dirname(HERE), "build", "obj" + suffix)
    os.makedirs(objdir, exist_ok=True)
    gendir = os.path.join(os.path.dirname(HERE), "build", "gen")
    os.makedirs(gendir, exist_ok=True)
    for src in RTC_SOURCES:
        text = open(os.path.join(CSRC, src)).read()
        assert ")QDEC_RTC\"" not in text
        with open(os.path.join(gendir, src.replace("_kernel.hip", "_src.inc")), "w") as fh:
            fh.write('R"QDEC_RTC(' + text + ')QDEC_RTC"\n')
    cflags = [f for f in FLAGS if f != "-shared"] + ["-I", gendir]

    def compile_one(src):
        obj = os.path.join(objdir, src + ".o")
        cmd = [_hipcc(), *cflags, *extra, "-c", "-o", obj, os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src} ({res.returncode}):\n{res.stderr[-6000:]}")
        if verbose and res.stderr:
            print(res.stderr[-4000:], file=sys.stderr)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 1), 16))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = lib + ".tmp"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", *link_flags, "-o", tmp, *objs,
           "-lhiprtc"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc link failed ({res.returncode}):\n{res.stderr[-6000:]}")
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    # python -m exp_ldpc_amd.build [--force] [--stamps] [--san] [--tag T -DNAME=V ...]
    argv = sys.argv[1:]
    tag = argv[argv.index("--tag") + 1] if "--tag" in argv else ""
    defs = [a[2:] for a in argv if a.startswith("-D")]
    san = "--san" in argv
    print(build(force="--force" in argv, verbose=True, stamps="--stamps" in argv, defines=defs, tag=tag,
                flags=SAN_FLAGS if san else (), link_flags=SAN_LINK if san else ()))
