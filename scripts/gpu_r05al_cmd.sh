set -o pipefail
mkdir -p gpurun_out/r05al
timeout -k 10 600 python -u -m pytest -x -v --durations=5 --timeout 500 --timeout-method thread -m gpu tests/test_vbhmm_hyp.py > gpurun_out/r05al/tests2.txt 2>&1
