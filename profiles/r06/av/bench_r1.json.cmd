# cmd: python bench.py --out gpurun_out/r06/av/bench_r1.json --no-cpu-baseline
