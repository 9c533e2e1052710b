#!/bin/bash
# Build variant libraries of the F(4x4) kernel (ablation flags in conv_winograd4.hip) next to the
# regular objects, for timing with tools/w4_layer.py --lib.  CPU-side; run before gpurun.
set -e
cd "$(dirname "$0")/.."
python -c "import __graft_entry__ as g; g.build()" >/dev/null
mkdir -p build/variants tools/wv
OBJS=$(python -c "
from facerecognitionpipeline_amd import build as b
import os
print(' '.join(os.path.join(b.BUILD, f'{src}.{b._digest(os.path.join(b.CSRC, src))}.o') for src in b.SOURCES if src != 'conv_winograd4.hip'))")
# VARIANTS: space-separated NAME or NAME:FLAG,FLAG (e.g. s55:W4_SPLIT0=5,W4_SPLIT1=5)
for E in ${VARIANTS:-base W4_NO_TRANSFORM W4_NO_PATCH W4_NO_ULOAD W4_NO_BARRIER}; do
  V=${E%%:*}; F=""; [ "$E" != "$V" ] && F=${E#*:}
  D=""; [ "$V" != base ] && [ -z "$F" ] && D="-D$V"
  [ -n "$F" ] && D=$(echo "$F" | tr ',' '\n' | sed 's/^/-D/' | tr '\n' ' ')
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $D -Iinclude -Ifacerecognitionpipeline_amd/csrc \
    -x hip -c facerecognitionpipeline_amd/csrc/conv_winograd4.hip -o build/variants/w4_$V.o &
done
wait
for E in ${VARIANTS:-base W4_NO_TRANSFORM W4_NO_PATCH W4_NO_ULOAD W4_NO_BARRIER}; do
  V=${E%%:*}
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,-rpath,/opt/rocm/lib build/variants/w4_$V.o $OBJS -o tools/wv/lib_$V.so
done
ls tools/wv/*.so
