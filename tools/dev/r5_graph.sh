# headline step eager vs replayed from a ring of HIP graphs, two passes each
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for gr in 0 1; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 --graph $gr --no-cpu-baseline --no-fg --no-intra --no-extra > gpurun_out/graph_$gr.json 2> gpurun_out/graph_$gr.err || { tail -5 gpurun_out/graph_$gr.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print('graph', sys.argv[2], d['value'], d['ms_per_step'], d.get('verified'))" gpurun_out/graph_$gr.json $gr
done; done
