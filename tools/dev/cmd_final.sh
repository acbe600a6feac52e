# round evidence: full GPU suite + smoke + bench + rocprof stats (gpu_check), then PMC traffic (gpu_profile)
set -o pipefail
TAG=${1:-r03s2}
timeout -k 10 1000 bash tools/gpu_check.sh $TAG || exit 1
timeout -k 10 1200 bash tools/gpu_profile.sh prof_$TAG
