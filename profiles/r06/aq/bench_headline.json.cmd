# cmd: python bench.py --out gpurun_out/r06/aq/bench_headline.json 
