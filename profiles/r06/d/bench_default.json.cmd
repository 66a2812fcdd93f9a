# cmd: python bench.py --out gpurun_out/r06/d/bench_default.json 
