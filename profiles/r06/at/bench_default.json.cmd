# cmd: python bench.py --out gpurun_out/r06/at/bench_default.json 
