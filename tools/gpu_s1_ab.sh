# stage-1 stride-2 conv2 tile A/B inside the forward: one-lane kernel traces of bench.py with the
# package build and tools/wv/lib_s1{a,b,c}.so; per-layer view offline (tools/prof_summary.py)
set -e
export TMPDIR=/tmp
O=gpurun_out/s1_ab
mkdir -p $O
cp facerecognitionpipeline_amd/libfrhip.so $O/base.so.keep
for v in base s1a s1b s1c base2; do
  case $v in base*) cp $O/base.so.keep facerecognitionpipeline_amd/libfrhip.so ;; *) cp tools/wv/lib_$v.so facerecognitionpipeline_amd/libfrhip.so ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --lanes-min 0 > $O/bench_$v.json 2> $O/bench_$v.err
done
cp $O/base.so.keep facerecognitionpipeline_amd/libfrhip.so
rm -f $O/base.so.keep
