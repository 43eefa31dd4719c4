set -e
for i in 1 2; do timeout -k 10 300 python tools/variant_bench.py --streams 2 --names ${AB_NAMES} -- ${AB_EXTRA:-}; done
