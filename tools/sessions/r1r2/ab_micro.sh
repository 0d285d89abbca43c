set -u
mkdir -p gpurun_out/ab_micro
for v in oldpk perm scbits; do
  NERFHIP_LIB=build/variants/v_$v.so timeout -k 10 240 python tools/bitwise_ab.py gpurun_out/ab_micro/bw_$v.npz > gpurun_out/ab_micro/bw_$v.log 2>&1 || { echo "bitwise $v failed"; tail -5 gpurun_out/ab_micro/bw_$v.log; exit 1; }
done
python tools/bitwise_ab.py --cmp gpurun_out/ab_micro/bw_oldpk.npz gpurun_out/ab_micro/bw_perm.npz
python tools/bitwise_ab.py --cmp gpurun_out/ab_micro/bw_oldpk.npz gpurun_out/ab_micro/bw_scbits.npz
AB_CONFIGS="medium:40 large:40 medium:1" bash tools/ab_run.sh micro build/variants/v_oldpk.so build/variants/v_perm.so build/variants/v_scbits.so
