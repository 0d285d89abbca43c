# A/B the row kernel's diagnostic variants (build/variants/v_*.so) on isolated groups.
set -e
for v in base NOSTAGE NOFLUSH; do
  lib=nerf-attention_amd/nerf_attention/_lib/libnerfhip.so
  [ $v != base ] && lib=build/variants/v_$v.so
  for c in "medium,deep,hifreq,lofreq --fits 160" "large --fits 40"; do
    echo "## $v $c"
    NERFHIP_LIB=$lib timeout -k 5 100 python tools/kbench.py --config $c --epochs 10 --precision bf16x3 --repeat 2 | grep rep
  done
done
