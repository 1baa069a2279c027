B="python -u bench.py --steps 20 --warmup 5 --no-legs --no-configs --no-cpu-baseline --iso-reps 3"
V=tools/variants_r06/mt32/liblodestar_bls.so
tools/gpu_steps.sh gpurun_out/r06k "timeout -k 10 240 $B" "LB_LIBRARY=$V timeout -k 10 240 $B" "LB_MSM_LANES=0 timeout -k 10 240 $B" "timeout -k 10 240 $B" "LB_LIBRARY=$V timeout -k 10 240 $B" "LB_MSM_LANES=0 timeout -k 10 240 $B"
