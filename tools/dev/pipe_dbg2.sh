set -o pipefail
echo "sync each"; MI_DBG_SYNC=1 timeout -k 10 200 python tools/dev/pipe_dbg.py 2>&1 | grep "^8 2" || exit 1
echo "spread"; MI_IR_SPREAD=1 timeout -k 10 200 python tools/dev/pipe_dbg.py 2>&1 | grep "^8 2" || exit 1
