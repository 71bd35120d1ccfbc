bash tools/quick32.sh && bash tools/run_variants_bench.sh && bash tools/run_stamps.sh
