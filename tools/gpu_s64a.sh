cd /root/repo && export TMPDIR=/tmp && o=gpurun_out/s64a && mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k gemm > $o/tests.log 2>&1; rc=$?; tail -3 $o/tests.log; [ $rc -ne 0 ] && { tail -40 $o/tests.log; exit $rc; }
timeout -k 10 300 python -u tools/gemm_libcmp.py vjepa2_amd/libvjepa_hip_stg32.so vjepa2_amd/libvjepa_hip.so > $o/cmp.log 2>&1; rc=$?; tail -4 $o/cmp.log; [ $rc -ne 0 ] && exit $rc
VJ_GEMM_STG=1 timeout -k 10 300 python -u tools/gemm_libcmp.py vjepa2_amd/libvjepa_hip_stg32.so vjepa2_amd/libvjepa_hip.so > $o/cmp_all.log 2>&1; rc=$?; tail -4 $o/cmp_all.log; [ $rc -ne 0 ] && exit $rc
TAG=s64a KCOLS="vjepa2_amd/libvjepa_hip_stg32.so vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_stg32.so@VJ_GEMM_STG=1 vjepa2_amd/libvjepa_hip.so@VJ_GEMM_STG=1" KIND=gemm ROUNDS=5 STEPS="VJ_LIB=vjepa2_amd/libvjepa_hip_stg32.so - VJ_GEMM_STG=1" RUNS=2 bash tools/gpu_ab.sh
