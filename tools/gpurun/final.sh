# the round's final measurement set on the committed build (tools/gpurun/run.sh steps)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_fuzz.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${1}_parity.log 2>&1 || { tail -5 gpurun_out/${1}_parity.log; exit 1; }
tail -1 gpurun_out/${1}_parity.log
bash tools/gpurun/run.sh $1 bench mixed prof profmixed pmc pmcmixed sq
