# headline with the chroma MC + chroma residual overlapped beside the luma residual, A/B (same box)
set -o pipefail
for rep in 1 2; do for f in "" --plane-overlap; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-fg --no-intra --no-extra --no-two-in-flight $f > gpurun_out/bpo.json 2> gpurun_out/bpo.err || { tail -5 gpurun_out/bpo.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/bpo.json'));print('overlap' if len(sys.argv) > 1 and sys.argv[1] else 'serial', d['value'], d['ms_per_step'], d.get('verified'))" "$f"
done; done
