# round-4: config-3 k_lloyd1 (compressed fp32 D = 3) SQ / TCC counter sets
bash tools/kernel_profile.sh gpurun_out/t10/pc_c3 k_lloyd1 --steps 20 --warmup 3 > gpurun_out/t10_pc_c3.txt 2>&1 || { tail -8 gpurun_out/t10_pc_c3.txt; exit 1; }
tail -42 gpurun_out/t10_pc_c3.txt | grep -E "k_lloyd1|k_upd|k_lists|SQ_|clock|frac|hbm|_ns"
