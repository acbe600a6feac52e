# round pass (GPU suite, smoke, bench) then the itx streaming-load A/B
set -o pipefail
bash tools/gpu_round.sh r05a || exit $?
STAGE=itx VARIANT=nt TESTS=tests/test_itx_gpu.py bash tools/dev/ab_stage.sh
