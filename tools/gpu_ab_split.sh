# A/B of a rebuilt libfrhip.so (package) against tools/wv/lib_base.so: head FC split-K sweep,
# serving latency and C3 bench, alternating builds on one box.  usage: bash tools/gpu_ab_split.sh
set -e
O=gpurun_out/ab_split
mkdir -p $O
for so in facerecognitionpipeline_amd/libfrhip.so tools/wv/lib_base.so; do
  n=$(basename $so .so)
  timeout -k 10 120 python -u tools/fc_sweep.py --so $so --tiles 8,3 --splits 32,49,98 > $O/fc_$n.txt 2>&1
  timeout -k 10 180 python -u tools/serve_latency.py --so $so > $O/serve_$n.txt 2>&1
done
cp facerecognitionpipeline_amd/libfrhip.so $O/new.so.keep
for i in 1 2; do
  cp $O/new.so.keep facerecognitionpipeline_amd/libfrhip.so
  timeout -k 10 240 python -u bench.py --no-cpu-baseline > $O/bench_new_$i.json 2>/dev/null
  cp tools/wv/lib_base.so facerecognitionpipeline_amd/libfrhip.so
  timeout -k 10 240 python -u bench.py --no-cpu-baseline > $O/bench_base_$i.json 2>/dev/null
done
rm -f $O/new.so.keep
