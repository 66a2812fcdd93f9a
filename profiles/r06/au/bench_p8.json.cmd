# cmd: python bench.py --out gpurun_out/r06/au/bench_p8.json --prompts 8 --no-cpu-baseline
