cd /root/repo && export TMPDIR=/tmp && o=gpurun_out/s64b && mkdir -p $o
for v in dm1 dm2; do VJ_GEMM_STG=1 timeout -k 10 300 python -u tools/gemm_libcmp.py vjepa2_amd/libvjepa_hip_stg32.so vjepa2_amd/libvjepa_hip_$v.so > $o/cmp_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 $o/cmp_$v.log)"; [ $rc -ne 0 ] && exit $rc; done
S=vjepa2_amd/libvjepa_hip
TAG=s64b KCOLS="${S}_stg32.so@VJ_GEMM_STG=1 ${S}.so@VJ_GEMM_STG=1 ${S}_dm1.so@VJ_GEMM_STG=1 ${S}_dm2.so@VJ_GEMM_STG=1" KIND=gemm ROUNDS=5 STEPS="VJ_LIB=${S}_stg32.so VJ_GEMM_STG=1 VJ_GEMM_STG=1,VJ_LIB=${S}_dm1.so VJ_GEMM_STG=1,VJ_LIB=${S}_dm2.so" RUNS=2 bash tools/gpu_ab.sh
