# round-4 combined evidence run: cold start (first GPU process), GPU tests, bench lines,
# proxies, counter sets (crowded, config 5), list-reuse budget sweep
bash tools/gpu_round4_t4.sh || exit 1
bash tools/gpu_round4_t5.sh || exit 1
