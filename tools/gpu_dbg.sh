set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "segments_equal or shared_prefix or lstm_backward_nonzero or encoder_backward_tail" 2>&1 | tail -25
