set -u
mkdir -p gpurun_out/pardma
for v in regstage pardma; do
  NERFHIP_LIB=build/variants/v_$v.so timeout -k 10 300 python tools/bitwise_ab.py gpurun_out/pardma/$v.npz 2>&1 | grep -v amdgpu.ids || exit 1
done
python tools/bitwise_ab.py --cmp gpurun_out/pardma/regstage.npz gpurun_out/pardma/pardma.npz
AB_CONFIGS="medium:40 large:40 small:40 tiny:40 large:5 medium:1" bash tools/ab_run.sh pardma build/variants/v_regstage.so build/variants/v_pardma.so > /dev/null
grep -v amdgpu.ids gpurun_out/ab_pardma/kbench.log | sed 's/"precision": "bf16x3", //; s/"rep": 0, //'
