set -o pipefail
mkdir -p gpurun_out
STAGE=deblock VARIANT=lfv TESTS=tests/test_lf_gpu.py bash tools/dev/ab_stage.sh
