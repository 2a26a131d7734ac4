set -u
mkdir -p gpurun_out
for v in default abl_load abl_store abl_both default; do
  if [ $v = default ]; then unset OFDM_MI355X_LIB; else export OFDM_MI355X_LIB=variants/libofdm_$v.so; fi
  echo -n "$v "; timeout -k 10 120 python tools/fft_ab.py 2>/dev/null || exit 3
done
