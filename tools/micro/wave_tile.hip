// Probe (r05): does a bigger per-wave output tile pay in the pair phases'
// main loop?  The pair phases stream each wave's 64-cout weight slice from L2
// into registers (4 x 1 KiB per 64-K step) and read the 16x16x64 B fragments
// from LDS; with two waves per SIMD a wave holds at most 256 registers, so its
// tile is 64 couts x 128 pixels and every weight byte serves 128 pixels
// (profiles/r05_diag_pair_weight_stream_probe.txt: the weight stream costs
// 13-16 % of the phases' cycles).  This loop models only the main loop:
//   T128: 512-thread workgroups (2 waves / SIMD), 64 x 128 tile, acc 128 VGPRs
//   T256: 256-thread workgroups (1 wave / SIMD, 512-register budget),
//         64 x 256 tile, acc 256 registers: half the weight bytes per MAC
// Same MFMA count per CU, same LDS B bytes per MAC, every wave a distinct
// weight slice (as conv5+6), weights 1.2 MB (L2-resident), random operands.
// Reports TOP/s, the in-kernel clock and cycles per 64-K step per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int S = 18;            // 64-K steps per tile (conv5: 128 cin x 9 taps / 64)
constexpr int COUT = 512;        // 8 distinct 64-cout slices
constexpr int WBUF = COUT * 64;  // bytes of one step's weight chunk

template <int NJ, int NT>
__global__ __launch_bounds__(NT, 1) void k(const int8_t* __restrict__ w, int* out, long long* clk, int tiles) {
  __shared__ __attribute__((aligned(16))) int lds[16384];   // 64 KB of random B bytes
  for (int i = threadIdx.x; i < 16384; i += NT) lds[i] = (int)(i * 2654435761u ^ blockIdx.x);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int p16 = lane & 15, g = lane >> 4;
  const int slice = (wave + blockIdx.x) & 7;
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(w), 0, 0x7fffffff, 0x00020000);
  const int voff = (slice * 64 + p16) * 64 + g * 16;
  const uint8_t* lb = reinterpret_cast<const uint8_t*>(lds) + lane * 16;
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  v4i acc[4][NJ];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < NJ; ++j) acc[i][j] = (v4i){0, 0, 0, 0};
  v4i ga[2][4];
  auto issue = [&](int s, int slot) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(wr, voff, s * WBUF + i * 1024, 0);
      ga[slot][i] = (v4i){(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
    }
  };
  auto rd_b = [&](int s, int j) {   // conflict-free lane-linear 1 KiB fragments
    return *reinterpret_cast<const v4i*>(lb + ((s * NJ + j) & 63) * 1024);
  };
  // B fragments through a 4-slot ring, each read 3 blocks ahead of its first
  // MFMA (block J = s * NJ + j, slot J % 4; S * NJ % 4 == 0 keeps the slots
  // continuous from tile to tile)
  static_assert((S * NJ) % 4 == 0, "ring continuity");
  v4i fb[4];
  issue(0, 0);
#pragma unroll
  for (int J = 0; J < 3; ++J) fb[J] = rd_b(0, J);
  for (int t = 0; t < tiles; ++t) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int J = s * NJ + j;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          __builtin_amdgcn_sched_barrier(0);
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ga[s & 1][i], fb[J & 3], acc[i][j], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          if (j == 0 && i == 1) {
            if (s + 1 < S) issue(s + 1, (s + 1) & 1);
            else issue(0, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        const int Jn = J + 3 < S * NJ ? J + 3 : J + 3 - S * NJ;
        fb[(J + 3) & 3] = rd_b(Jn / NJ, Jn % NJ);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  int x = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < NJ; ++j) x += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  out[blockIdx.x * NT + threadIdx.x] = x;
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

template <int NJ, int NT>
static void run(const char* name, const int8_t* w, int* out, long long* clk, int ncu) {
  const int tiles = 8 * 256 / (NJ * (NT / 64)) * 8;   // same MFMAs per CU for both forms
  for (int rep = 0; rep < 4; ++rep) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k<NJ, NT>), dim3(ncu), dim3(NT), 0, 0, w, out, clk, tiles);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(ncu * 2);
    (void)hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> ghz;
    double cyc = 0;
    for (int b = 0; b < ncu; ++b) {
      ghz.push_back(h[2 * b] / (double)h[2 * b + 1] * 0.1);
      cyc += h[2 * b];
    }
    std::sort(ghz.begin(), ghz.end());
    const double macs = (double)ncu * (NT / 64) * tiles * S * 4 * NJ * 16 * 16 * 64;
    const double steps = (double)tiles * S;
    if (rep > 0)
      printf("%-44s %.3f ms  %.0f TOP/s  clock %.3f GHz  %.0f cyc per 64-K step per wave (%d MFMA = %d issue cyc)\n",
             name, ms, 2 * macs / (ms * 1e-3) / 1e12, ghz[ghz.size() / 2], cyc / ncu / steps, 4 * NJ, 4 * NJ * 16);
    fflush(stdout);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
}

int main() {
  int dev = 0, ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int8_t* w;
  int* out;
  long long* clk;
  const size_t wbytes = (size_t)S * WBUF;
  (void)hipMalloc(&w, wbytes);
  (void)hipMalloc(&out, (size_t)ncu * 512 * 4);
  (void)hipMalloc(&clk, (size_t)ncu * 16);
  std::vector<int8_t> hw(wbytes);
  for (size_t i = 0; i < wbytes; ++i) hw[i] = (int8_t)(i * 2654435761u >> 13);
  (void)hipMemcpy(w, hw.data(), wbytes, hipMemcpyHostToDevice);
  printf("%d CUs, weights %.2f MB\n", ncu, wbytes / 1e6);
  for (int pass = 0; pass < 2; ++pass) {
    run<8, 512>("T128: 8 waves/CU, 64x128 tile per wave", w, out, clk, ncu);
    run<16, 256>("T256: 4 waves/CU, 64x256 tile per wave", w, out, clk, ncu);
  }
  return 0;
}
