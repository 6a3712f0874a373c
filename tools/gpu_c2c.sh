#!/bin/bash
# Config 2 standalone under the bench's conditions: hardware queues, other contexts with big batches.
set -o pipefail
echo "plain: $(timeout -k 10 120 python tools/config2_run.py 40)" || exit 1
echo "hwq8: $(GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python tools/config2_run.py 40)" || exit 1
echo "busy4: $(C2_BUSY=4 timeout -k 10 200 python tools/config2_run.py 40)" || exit 1
echo "hwq8+busy4: $(GPU_MAX_HW_QUEUES=8 C2_BUSY=4 timeout -k 10 200 python tools/config2_run.py 40)" || exit 1
