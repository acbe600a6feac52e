set -o pipefail
for rep in 1 2; do for g in 0 1; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-fg --no-intra --no-extra --graph $g > gpurun_out/g$g.json 2> gpurun_out/g$g.err || { tail -5 gpurun_out/g$g.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/g$g.json')); print('graph=$g', d['value'], d['ms_per_step'], d['verified'])"
done; done
