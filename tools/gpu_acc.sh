set -o pipefail
echo "== x3"; timeout -k 10 120 python tools/lstm_accuracy.py || exit 1
echo "== f32"; SGG_LIB=$PWD/tools/abx/libsgg_f32.so timeout -k 10 120 python tools/lstm_accuracy.py || exit 1
echo "== bwd probe"; timeout -k 10 60 tools/run/lstm_bwd_probe 2560 20 || exit 1
