set -e
mkdir -p gpurun_out/c4p
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c4p/on.json 2> gpurun_out/c4p/on.err
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline --c4-pipeline off > gpurun_out/c4p/off.json 2> gpurun_out/c4p/off.err
