# headline with and without the two-in-flight extra pipeline, alternating (same box)
set -o pipefail
for rep in 1 2; do for f in --two-in-flight --no-two-in-flight; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fg --no-intra --no-extra $f > gpurun_out/b2if.json 2>/dev/null || exit 1
  python -c "import json,sys;d=json.load(open('gpurun_out/b2if.json'));print(sys.argv[1], d['value'], d['ms_per_step'], (d['two_frames_in_flight'] or {}).get('value'))" -- $f
done; done
