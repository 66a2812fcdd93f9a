# cmd: python bench.py --out gpurun_out/r06/k/bench_headline.json 
