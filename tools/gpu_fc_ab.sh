# head-FC tile A/B inside the forward: kernel traces of bench.py (one lane) with the package
# build and with tools/wv/lib_fc64.so (the FC of <= 256 rows on 64x128), per-layer view offline
set -e
export TMPDIR=/tmp
O=gpurun_out/fc_ab
mkdir -p $O
cp facerecognitionpipeline_amd/libfrhip.so $O/base.so.keep
for v in base fc64 base2; do
  if [ $v = fc64 ]; then cp tools/wv/lib_fc64.so facerecognitionpipeline_amd/libfrhip.so; else cp $O/base.so.keep facerecognitionpipeline_amd/libfrhip.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --lanes-min 0 > $O/bench_$v.json 2> $O/bench_$v.err
  timeout -k 10 240 python3 bench.py --no-cpu-baseline > $O/b2_$v.json 2>/dev/null
done
rm -f $O/base.so.keep
