// Device probe for the lazy 28-bit G2 chain and the dedicated squaring (diagnostic, not product):
// kernel 1 runs only the squaring-based exponentiations, kernel 2 only the lazy [|x|]Q chain and
// compares it with the canonical Fp2 chain on the device.  Each launch is synchronised and checked.
#include "../lodestar_amd/csrc/curve.h"
#include <cstdio>
#include <cstring>
#include <cstdlib>
using namespace gbv;

static const char* HEX[2][4] = {
  {"024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8",
   "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e",
   "0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801",
   "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be"},
  {"00c85d5ad55709df9f7add6bbc1dab8537bca1f7a08dda2803047fb0ec79bc4fb114440efcc4459cb41400ed6d01d98c",
   "00b383ec2171a4820ffb284d92c5c046080227eb5b60ed71db04d7d0e78fb20889f265ae5e061669811569a6a6c4918a",
   "148b911d5344771d62d920b03cd0b46e1a1e58c02eea292d068c59b6a20e73726f24bb5323dbcf1322299d5bb8cca539",
   "015973f0ea10e3a66091f305bf042d84688a13c9baefc6cef4d83bf1e34b66b205d53d208d0748fc3e6e09eb2e1ea694"}};

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_probe_sqr(uint32_t* ok) {
  Fp y = fp_zero();
  y.v[0] = 3 + threadIdx.x;
  y = fp_to_mont(y);
  Fp y2 = fp_sqr(y);
  Fp r = fp_sqrt_candidate(y2);
  ok[threadIdx.x] = fp_eq(fp_sqr(r), y2) && fp_eq(fp_mul(y, y), y2);
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_probe_lazy(const uint8_t* pts, uint32_t* ok, uint32_t nact) {
  if (threadIdx.x >= nact) return;
  const uint8_t* b = pts + 192 * (threadIdx.x & 1);
  G2A q{Fp2{fp_to_mont(fp_load_be48(b, false)), fp_to_mont(fp_load_be48(b + 48, false))},
        Fp2{fp_to_mont(fp_load_be48(b + 96, false)), fp_to_mont(fp_load_be48(b + 144, false))}};
  G2J l = g2_mul_xabs_lazy(q), r = g2_mul_xabs(q);
  Fp2 z1 = fp2_sqr(l.z), z2 = fp2_sqr(r.z);
  bool same = fp2_eq(fp2_mul(l.x, z2), fp2_mul(r.x, z1)) &&
              fp2_eq(fp2_mul(l.y, fp2_mul(z2, r.z)), fp2_mul(r.y, fp2_mul(z1, l.z)));
  ok[threadIdx.x] = (same ? 1u : 0u) | (g2_in_subgroup(q) ? 2u : 0u);
}

static int check(hipError_t e, const char* what) {
  if (e != hipSuccess) { printf("%s: %s\n", what, hipGetErrorString(e)); return 1; }
  return 0;
}

int main(int argc, char** argv) {
  uint8_t pts[384];
  for (int p = 0; p < 2; ++p)
    for (int c = 0; c < 4; ++c)
      for (int i = 0; i < 48; ++i) {
        unsigned v;
        sscanf(HEX[p][c] + 2 * i, "%2x", &v);
        pts[192 * p + 48 * c + i] = (uint8_t)v;
      }
  uint8_t* dp; uint32_t* dok; uint32_t ok[64];
  if (check(hipMalloc(&dp, 384), "malloc") || check(hipMalloc(&dok, 256), "malloc")) return 1;
  hipMemcpy(dp, pts, 384, hipMemcpyHostToDevice);
  const bool want_lazy = argc < 2 || strcmp(argv[1], "sqr") != 0;
  k_probe_sqr<<<1, 64>>>(dok);
  if (check(hipDeviceSynchronize(), "k_probe_sqr")) return 1;
  hipMemcpy(ok, dok, 256, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) bad += ok[i] != 1;
  printf("k_probe_sqr: %d/64 lanes consistent\n", 64 - bad);
  if (!want_lazy) return bad != 0;
  const uint32_t nact = argc > 2 ? (uint32_t)atoi(argv[2]) : 64;
  hipMemset(dok, 0, 256);
  k_probe_lazy<<<1, 64>>>(dp, dok, nact);
  if (check(hipDeviceSynchronize(), "k_probe_lazy")) return 1;
  hipMemcpy(ok, dok, 256, hipMemcpyDeviceToHost);
  int bad2 = 0;
  for (int i = 0; i < (int)nact; ++i) bad2 += ok[i] != ((i & 1) ? 1u : 3u);
  printf("k_probe_lazy: %d/%u lanes as expected (lane0 %u lane1 %u)\n", (int)nact - bad2, nact, ok[0], ok[1]);
  return (bad || bad2) ? 1 : 0;
}
