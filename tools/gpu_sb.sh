cd /root/repo && export TMPDIR=/tmp && o=gpurun_out/sb && mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "gemm or gelu" > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -ne 0 ] && { tail -30 $o/tests.log; exit $rc; }
for c in "fc2  tgt bf16" "qkv  tgt"; do VJ_STAMPS_LIB=vjepa2_amd/libvjepa_hip_stamps.so timeout -k 10 120 python -u tools/gemm_stamps.py "$c" 2>&1 | grep -v "amdgpu.ids\|spread" || exit 3; done
TAG=sb KCOLS="vjepa2_amd/libvjepa_hip_sb4.so vjepa2_amd/libvjepa_hip_sb5.so vjepa2_amd/libvjepa_hip.so" KIND=gemm ROUNDS=5 STEPS="VJ_LIB=vjepa2_amd/libvjepa_hip_sb4.so VJ_LIB=vjepa2_amd/libvjepa_hip_sb5.so -" RUNS=2 bash tools/gpu_ab.sh
