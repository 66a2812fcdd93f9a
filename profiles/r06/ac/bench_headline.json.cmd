# cmd: python bench.py --out gpurun_out/r06/ac/bench_headline.json 
