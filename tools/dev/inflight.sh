set -o pipefail
mkdir -p gpurun_out
for cfg in "1 0" "2 0" "2 1" "3 1" "4 1" "2 0"; do
set -- $cfg
timeout -k 10 200 python bench.py --no-cpu-baseline --no-fg --no-intra --no-extra --no-verify --inflight $1 --stagger $2 --steps 40 > gpurun_out/infl.json 2> gpurun_out/infl.err || { tail -5 gpurun_out/infl.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/infl.json')); print('$cfg', d['value'], d['ms_per_step'], d['fps'])"
done
