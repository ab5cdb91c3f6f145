// Latency calibration on one wave (gfx950): dependent FP64 FMA, FP64 add, DPP-move + add, LDS read
// (pointer chase), global read hitting L2 (pointer chase), v_readlane round trip, FP64 division and
// sqrt, each as shader-clock cycles per dependent step.  Build: hipcc -O3 --offload-arch=gfx950
// tools/dbg/latency_calib.hip -o tools/dbg/latency_calib ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int kSteps = 4096;

__global__ void k_calib(double* out, const int* chain, double x0, unsigned long long* cyc) {
  __shared__ int lchain[1024];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) lchain[i] = chain[i];
  __syncthreads();
  double x = x0 + lane * 1e-9;
  unsigned long long t0, t1;
  // 1. FP64 fma chain
  t0 = clock64();
  for (int i = 0; i < kSteps; ++i) x = fma(x, 0.999999, 1e-7);
  t1 = clock64();
  if (lane == 0) cyc[0] = t1 - t0;
  // 2. FP64 add chain
  t0 = clock64();
  for (int i = 0; i < kSteps; ++i) x = x + 1e-9;
  t1 = clock64();
  if (lane == 0) cyc[1] = t1 - t0;
  // 3. DPP (quad_perm xor 1) on both halves + add
  t0 = clock64();
  for (int i = 0; i < kSteps; ++i) {
    union { double d; int v[2]; } u, r;
    u.d = x;
    r.v[0] = __builtin_amdgcn_update_dpp(0, u.v[0], 0xB1, 0xF, 0xF, false);
    r.v[1] = __builtin_amdgcn_update_dpp(0, u.v[1], 0xB1, 0xF, 0xF, false);
    x = x + r.d * 1e-3;
  }
  t1 = clock64();
  if (lane == 0) cyc[2] = t1 - t0;
  // 4. LDS pointer chase
  int p = lane;
  t0 = clock64();
  for (int i = 0; i < kSteps; ++i) p = lchain[p & 1023];
  t1 = clock64();
  if (lane == 0) cyc[3] = t1 - t0;
  // 5. global pointer chase (L2-resident 4 KB table)
  int q = lane;
  t0 = clock64();
  for (int i = 0; i < 512; ++i) q = __builtin_nontemporal_load(chain + (q & 1023));
  t1 = clock64();
  if (lane == 0) cyc[4] = (t1 - t0) * (kSteps / 512);
  // 6. readlane round trip: value -> SGPR -> VALU
  t0 = clock64();
  for (int i = 0; i < kSteps; ++i) {
    union { double d; int v[2]; } u;
    u.d = x;
    u.v[0] = __builtin_amdgcn_readlane(u.v[0], 5);
    u.v[1] = __builtin_amdgcn_readlane(u.v[1], 5);
    x = u.d * 0.9999999 + 1e-9;
  }
  t1 = clock64();
  if (lane == 0) cyc[5] = t1 - t0;
  // 7. FP64 division chain
  t0 = clock64();
  for (int i = 0; i < kSteps; ++i) x = 1.0 + 1.0 / (x + 2.0);
  t1 = clock64();
  if (lane == 0) cyc[6] = t1 - t0;
  // 8. FP64 sqrt chain
  t0 = clock64();
  for (int i = 0; i < kSteps; ++i) x = sqrt(x + 1.0);
  t1 = clock64();
  if (lane == 0) cyc[7] = t1 - t0;
  // 9. erfc chain
  t0 = clock64();
  for (int i = 0; i < kSteps / 8; ++i) x = 1.0 + erfc(x - 1.5);
  t1 = clock64();
  if (lane == 0) cyc[8] = (t1 - t0) * 8;
  // 10. log chain
  t0 = clock64();
  for (int i = 0; i < kSteps / 8; ++i) x = 2.0 + log(x);
  t1 = clock64();
  if (lane == 0) cyc[9] = (t1 - t0) * 8;
  out[lane] = x + p + q;
}

int main() {
  std::vector<int> chain(1024);
  for (int i = 0; i < 1024; ++i) chain[i] = (i * 97 + 13) & 1023;
  int* dchain;
  double* dout;
  unsigned long long* dcyc;
  hipMalloc(&dchain, 1024 * sizeof(int));
  hipMalloc(&dout, 64 * sizeof(double));
  hipMalloc(&dcyc, 16 * sizeof(unsigned long long));
  hipMemcpy(dchain, chain.data(), 1024 * sizeof(int), hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k_calib, dim3(1), dim3(64), 0, 0, dout, dchain, 0.5, dcyc);
  hipDeviceSynchronize();
  unsigned long long cyc[16];
  hipMemcpy(cyc, dcyc, sizeof(cyc), hipMemcpyDeviceToHost);
  const char* names[] = {"fma_f64", "add_f64", "dpp2+add", "lds_chase", "global_chase", "readlane2+fma",
                         "div_f64", "sqrt_f64", "erfc_f64", "log_f64"};
  printf("{");
  for (int i = 0; i < 10; ++i) printf("%s\"%s\": %.1f", i ? ", " : "", names[i], (double)cyc[i] / kSteps);
  printf("}\n");
  return 0;
}
