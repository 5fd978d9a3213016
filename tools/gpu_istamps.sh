cd /root/repo && export TMPDIR=/tmp
for c in "qkv  tgt" "fc2  tgt bf16" "fc1  tgt" "dgrad fc2 Wt"; do
  VJ_GEMM_STG=1 VJ_STAMPS_LIB=vjepa2_amd/libvjepa_hip_stamps.so timeout -k 10 120 python -u tools/gemm_stamps.py "$c" 2>&1 | grep -v "amdgpu.ids\|spread" || exit 3
done
