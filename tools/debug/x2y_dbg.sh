# x2y / x2 bit-exactness at the grids where the store-data hazard showed (then the full
# C2 digest with every variant pinned).
set -e
CASES="4096x2048:1 4096x2048:3 4096x4096:2 2048x4096:2" SEGS="64 96" timeout -k 10 200 python -u tools/debug/x2y_diff.py
KERN=x2 CASES="4096x2048:3 4096x4096:2" SEGS="64" timeout -k 10 120 python -u tools/debug/x2y_diff.py
KERNELS="auto x2y x2" timeout -k 10 200 python -u tools/debug/digest_variants.py
