# fb_bwd4_kernel with two quads per wave at 3 waves per SIMD (q2w3, 168 VGPRs) on the
# round-4 step: C4 and 12,500-base A/B, parity sample
set -o pipefail
OUT=gpurun_out/r04s; mkdir -p $OUT
PARITY=1 timeout -k 10 900 bash scripts/ab_lib.sh build/ab/q2w3.so > $OUT/ab_c4.txt 2>&1; cat $OUT/ab_c4.txt
timeout -k 10 600 bash scripts/ab_lib.sh --args "--N 12500 --steps 40 --warmup 5" build/ab/q2w3.so > $OUT/ab_12k.txt 2>&1; cat $OUT/ab_12k.txt
