// Probe: v_dot2c_f32_bf16 as an exact residual v - bf16 half (update_kernels.hip sub_bf16_lo/hi).
// Prints mismatches against the plain fp32 subtraction for the inline-constant form the compiler
// picks and for the constant held in a register; then the register form on special
// inputs: a finite value whose pair partner is +-inf or NaN (h.hi * 0 = NaN spreads into the finite
// value's residual), and fp32 denormal / bf16-denormal values (whether the dot2 flushes them).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__global__ void k(const float* v, float* o, uint32_t cl, uint32_t ch, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = v[2 * i], b = v[2 * i + 1];
  const bf16x2_t p = {(__bf16)a, (__bf16)b};
  const uint32_t h = __builtin_bit_cast(uint32_t, p);
  o[4 * i + 0] = __builtin_amdgcn_fdot2_f32_bf16(p, __builtin_bit_cast(bf16x2_t, 0x0000BF80u), a, false);
  o[4 * i + 1] = __builtin_amdgcn_fdot2_f32_bf16(p, __builtin_bit_cast(bf16x2_t, 0xBF800000u), b, false);
  o[4 * i + 2] = __builtin_amdgcn_fdot2_f32_bf16(p, __builtin_bit_cast(bf16x2_t, cl), a, false);
  o[4 * i + 3] = __builtin_amdgcn_fdot2_f32_bf16(p, __builtin_bit_cast(bf16x2_t, ch), b, false);
  (void)h;
}
int main() {
  const int n = 1 << 16;
  std::mt19937 g(1);
  std::normal_distribution<float> d(0.f, 1.f);
  float* hv = new float[2 * n];
  for (int i = 0; i < 2 * n; ++i) hv[i] = d(g) * (i % 7 == 0 ? 1e-3f : 1.f);
  float *dv, *dout;
  hipMalloc(&dv, 8 * n);
  hipMalloc(&dout, 16 * n);
  hipMemcpy(dv, hv, 8 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dv, dout, 0x0000BF80u, 0xBF800000u, n);
  float* ho = new float[4 * n];
  hipMemcpy(ho, dout, 16 * n, hipMemcpyDeviceToHost);
  int bad[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < 2; ++j) {
      const float x = hv[2 * i + j];
      uint32_t u;
      memcpy(&u, &x, 4);
      const uint32_t r = u + 0x7FFFu + ((u >> 16) & 1u);  // round to nearest even bf16
      uint32_t hb = r & 0xFFFF0000u;
      float hf;
      memcpy(&hf, &hb, 4);
      const float want = x - hf;
      for (int form = 0; form < 2; ++form) {
        const float got = ho[4 * i + 2 * form + j];
        if (memcmp(&got, &want, 4) != 0) {
          if (bad[2 * form + j] < 3) printf("form %d half %d: v=%a want %a got %a\n", form, j, x, want, got);
          ++bad[2 * form + j];
        }
      }
    }
  }
  printf("mismatches: inline lo %d, literal hi %d, register lo %d, register hi %d (of %d each)\n", bad[0], bad[1], bad[2], bad[3], n);
  // special inputs, register form only: [finite, partner] pairs
  const float inf = __builtin_inff(), qnan = __builtin_nanf("");
  const float specials[][2] = {{1.5f, inf}, {1.5f, -inf}, {1.5f, qnan}, {inf, 1.5f}, {qnan, 1.5f},
                               {1e-39f, 1.0f}, {1.0f, 1e-39f}, {3e-39f, -2e-40f}, {1.17549435e-38f, 1.0f},
                               {1.2e-38f * 1.001f, 2.5f}};
  const int ns = sizeof(specials) / sizeof(specials[0]);
  float* hs = new float[2 * 256]();
  for (int i = 0; i < ns; ++i) { hs[2 * i] = specials[i][0]; hs[2 * i + 1] = specials[i][1]; }
  hipMemcpy(dv, hs, 8 * 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, dv, dout, 0x0000BF80u, 0xBF800000u, 256);
  hipMemcpy(ho, dout, 16 * 256, hipMemcpyDeviceToHost);
  for (int i = 0; i < ns; ++i) {
    for (int j = 0; j < 2; ++j) {
      const float x = hs[2 * i + j];
      uint32_t u;
      memcpy(&u, &x, 4);
      const uint32_t r = u + 0x7FFFu + ((u >> 16) & 1u);
      uint32_t hb = (u & 0x7F800000u) == 0x7F800000u ? u : (r & 0xFFFF0000u);
      float hf;
      memcpy(&hf, &hb, 4);
      const float want = x - hf, got = ho[4 * i + 2 + j];
      printf("special pair (%a, %a) half %d: v - bf16(v) want %a got %a%s\n", hs[2 * i], hs[2 * i + 1], j, want, got,
             memcmp(&got, &want, 4) ? "  <- differs" : "");
    }
  }
  return (bad[0] + bad[1] + bad[2] + bad[3]) ? 1 : 0;
}
