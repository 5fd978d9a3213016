// Measured MI355X peaks for the roofline denominators: dense MFMA throughput for
// the instructions the kernels issue (bf16 16x16x32 / 32x32x16, scaled fp8 16x16x128) and HBM
// read / copy bandwidth. Registers-only MFMA loops (no LDS, no memory) on every CU; the clock is
// whatever the card's power management gives under that load, which is the point.
// build: hipcc --offload-arch=gfx950 -O3 tools/peak.hip -o tools/peak_bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float fx4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int NACC = 8;

__global__ __launch_bounds__(256) void k_bf16_16(int iters, float* out) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = (__bf16)(0.002f * i);
  }
  f32x4 acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = f32x4{(float)j, 0.f, 0.f, (float)threadIdx.x};  // distinct: no CSE
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int j = 0; j < NACC; ++j)  // asm: the accumulators stay put (the builtin form got register-shuffled)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[j]) : "v"(a), "v"(b));
  float s = 0.f;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_bf16_32(int iters, float* out) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (threadIdx.x + i));
    b[i] = (__bf16)(0.002f * i);
  }
  f32x16 acc[4];
  for (int j = 0; j < 4; ++j)
    for (int r = 0; r < 16; ++r) acc[j][r] = (float)(j + r);
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
  float s = 0.f;
  for (int j = 0; j < 4; ++j)
    for (int r = 0; r < 16; ++r) s += acc[j][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fp8_16(int iters, float* out) {
  i32x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = 0x38383838 + threadIdx.x;
    b[i] = 0x30303030 + i;
  }
  f32x4 acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = f32x4{(float)j, 0.f, 0.f, (float)threadIdx.x};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int j = 0; j < NACC; ++j)
      acc[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[j], 0, 0, 0, 127, 0, 127);
  float s = 0.f;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_read(const fx4* __restrict__ src, long n, float* out) {
  fx4 s = {0.f, 0.f, 0.f, 0.f};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    fx4 v = __builtin_nontemporal_load(src + i);
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  if (s.x + s.y + s.z + s.w == 1234.5f) out[0] = s.x;  // keeps the loads
}

__global__ __launch_bounds__(256) void k_copy(const fx4* __restrict__ src, fx4* __restrict__ dst, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

template <class F>
static float time_ms(F f, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  f();  // warm (clocks, code load)
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) f();
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipGetLastError());
  return ms / reps;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_mhz_max\": %d", p.gcnArchName, cus, p.clockRate / 1000);
  float* out;
  CHECK(hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float)));
  const int blocks = cus * 8;  // 8 blocks x 4 waves per CU: 8 waves per SIMD
  const int iters = 20000;
  {
    float ms = time_ms([&] { k_bf16_16<<<blocks, 256>>>(iters, out); }, 5);
    double fl = (double)blocks * 4 * iters * NACC * 16 * 16 * 32 * 2;
    printf(", \"bf16_16x16x32_tflops\": %.1f", fl / ms / 1e9);
  }
  {
    float ms = time_ms([&] { k_bf16_32<<<blocks, 256>>>(iters, out); }, 5);
    double fl = (double)blocks * 4 * iters * 4 * 32 * 32 * 16 * 2;
    printf(", \"bf16_32x32x16_tflops\": %.1f", fl / ms / 1e9);
  }
  {
    float ms = time_ms([&] { k_fp8_16<<<blocks, 256>>>(iters, out); }, 5);
    double fl = (double)blocks * 4 * iters * NACC * 16 * 16 * 128 * 2;
    printf(", \"fp8_16x16x128_tflops\": %.1f", fl / ms / 1e9);
  }
  {
    const long bytes = 4L << 30;
    fx4 *src, *dst;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&dst, bytes));
    CHECK(hipMemset(src, 0, bytes));
    const long n = bytes / 16;
    float ms = time_ms([&] { k_read<<<cus * 16, 256>>>(src, n, out); }, 10);
    printf(", \"hbm_read_gbs\": %.0f", bytes / ms / 1e6);
    ms = time_ms([&] { k_copy<<<cus * 16, 256>>>(src, dst, n); }, 10);
    printf(", \"hbm_copy_gbs\": %.0f", 2.0 * bytes / ms / 1e6);
    CHECK(hipFree(src));
    CHECK(hipFree(dst));
  }
  printf("}\n");
  CHECK(hipFree(out));
  return 0;
}
