# detector tile-rule A/B: fr_detect time of the package build vs tools/wv/lib_<v>.so variants
set -e
O=gpurun_out/det_ab
mkdir -p $O
: > $O/det.txt
for so in "" tools/wv/lib_dA.so tools/wv/lib_dB.so tools/wv/lib_dC.so ""; do
  timeout -k 10 120 python -u tools/det_time.py ${so:+--so $so} >> $O/det.txt 2>/dev/null
done
