set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r02_c2.json 2> gpurun_out/r02_c2.err && \
timeout -k 10 200 python bench.py --config c4 --steps 10 --warmup 2 > gpurun_out/r02_c4.json 2> gpurun_out/r02_c4.err && \
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --sustain-frames 0 > gpurun_out/r02_c5.json 2> gpurun_out/r02_c5.err && \
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --sustain-frames 0 > gpurun_out/r02_c3.json 2> gpurun_out/r02_c3.err
