# cmd: python bench.py --out gpurun_out/r06/au/bench_p8b.json --prompts 8 --no-cpu-baseline
