set -eo pipefail
O=gpurun_out/r06c5b; mkdir -p $O
F="--no-cpu-baseline --no-c4 --no-reference-default --no-c3 --no-sample-phase --variant none --steps 3"
for cfg in "new:" "old:--ssf-streams 0 --stream-priority 0" "new2:"; do
  name=${cfg%%:*}; flags=${cfg#*:}
  timeout -k 10 400 python -u bench.py $F $flags --detail-out $O/$name.detail.json > $O/$name.json 2> $O/$name.err
  python -c "import json; d=json.load(open('$O/$name.json')); print('$name', round(d['value']/1e6,2), d['configs']['c5']['shots_per_s'])"
done
