# C4 bench twice (detections must agree run to run now that the frames are seeded) + detector timing
set -e
O=gpurun_out/c4s
mkdir -p $O
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > $O/c4_1.json 2>/dev/null
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > $O/c4_2.json 2>/dev/null
timeout -k 10 120 python -u tools/det_time.py > $O/det.txt 2>/dev/null
timeout -k 10 120 python -u tools/det_time.py >> $O/det.txt 2>/dev/null
