# round evidence: full GPU suite + smoke + bench + rocprof stats (gpu_check), PMC traffic
# (gpu_profile), then the bench with two frames in flight
set -o pipefail
TAG=${1:-r03s2}
timeout -k 10 1000 bash tools/gpu_check.sh $TAG || exit 1
timeout -k 10 1200 bash tools/gpu_profile.sh prof_$TAG || exit 1
timeout -k 10 300 python bench.py --two-in-flight --no-cpu-baseline --no-fg --no-intra --no-extra > gpurun_out/two_$TAG.json 2> gpurun_out/two_$TAG.err
