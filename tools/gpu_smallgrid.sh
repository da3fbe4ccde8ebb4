set -e
echo "== default"; timeout -k 10 120 python tools/enc_bench.py
echo "== V2_SMALL=0"; timeout -k 10 120 python tools/enc_bench.py --tune 9=0
echo "== V4_SPLITK=0 (no split)"; timeout -k 10 120 python tools/enc_bench.py --tune 6=0
