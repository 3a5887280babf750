// MFMA GEMMs for libwhisper_hip.
//
//   Y[m][n] = sum_k X[m][k] * W[n][k]        (W in nn.Linear [out][in] layout)
//
// Two kernels:
//   * k_gemm_tile  — 128x128 output tiles, LDS double buffer, register-staged
//     global loads; used where M is large (encoder blocks, conv1/conv2 as
//     overlapping-row im2col views, cross-KV precompute, long prefills).
//     MFMA-bound: 2*M*N*K flop per call.
//   * k_gemv_rows  — "skinny" weight-streaming GEMM for M <= 128 rows (decoder
//     step at W windows x B beams, short prefills, vocab projection).  One
//     workgroup = 16 output columns x all rows, its 8 waves split K; weights are
//     streamed from HBM exactly once.  HBM-bound: N*K*sizeof(T) bytes per call.
//
// Both use the swapped product D^T = W * X^T so each lane ends with 4
// consecutive output columns of one row (wide epilogue stores).
#include "wh_gemm.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>

namespace wh {

// ============================================================ big tile GEMM
constexpr int TBM = 128, TBN = 128, TKB = 128;  // TKB = bytes of K per tile row
constexpr int TROW = TKB + 16;                  // padded LDS row stride (bytes): conflict-free b128 reads

// TBN_ = 128 or 64 output columns per tile (64: grids below one tile per CU, e.g. the
// n-wide encoder GEMMs of a single window: 120 -> 240 workgroups).
// KZ = 2 (round 4, the single-window encoder's residual GEMMs): each tile's K is split in
// two halves run by two workgroups (480 for 240 tiles: two per CU), which meet per wave in
// the launch: each wave stores its fp32 sub-tile write-through (sc1) into a.p1_slab,
// drains it, adds to the (tile, wave) counter (relaxed agent atomic); the second arriver
// re-arms the counter, loads the other half with sc1 loads and adds: acc + other, which is
// the same bits whichever half arrives last (fp32 addition commutes), then the epilogue.
template <typename T, int EPI, int TBN_ = TBN, int KZ = 1>
__global__ __launch_bounds__(256, 2) void k_gemm_tile(GemmArgs a) {
  static_assert(KZ == 1 || KZ == 2, "two K halves at most (their sum commutes)");
  constexpr int BK = TKB / (int)sizeof(T);  // 64 half / 32 float
  constexpr int KS = BK / 32;               // k-steps per tile
  constexpr int WCH = TBN_ / 32;            // W chunks per thread (TBN_ rows x 8 chunks / 256)
  constexpr int NI = TBN_ / 32;             // 16-column fragments per wave (wave tile 64 x TBN_/2)
  __shared__ __attribute__((aligned(16))) char smem[2][(TBM + TBN_) * TROW];  // [buf][X rows | W rows]

  const int ntn = a.N / TBN_;
  const int ntm = (a.M + TBM - 1) / TBM;
  // the KZ halves of a tile are neighbours in the remapped order (same XCD)
  const int rid = xcd_remap(blockIdx.x, ntm * ntn * KZ);
  const int bid = rid / KZ, kz = rid - bid * KZ;
  const int tm = bid / ntn, tn = bid % ntn;
  const int m0 = tm * TBM, n0 = tn * TBN_;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int r = lane & 15, g = lane >> 4;

  const T* X = reinterpret_cast<const T*>(a.X);
  const T* W = reinterpret_cast<const T*>(a.W);

  // per-thread global source rows of its 16 B chunks (8 per row): 4 of X, WCH of W
  const char* xsrc[4];
  const char* wsrc[WCH];
  int lds_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    const int row = c >> 3, col = c & 7;
    int m = m0 + row;
    if (m >= a.M) m = a.M - 1;
    const int gi = m / a.x_group_rows, ri = m - gi * a.x_group_rows;
    const int64_t k0 = (int64_t)kz * (a.K / KZ);  // this workgroup's K half
    xsrc[i] = reinterpret_cast<const char*>(X + (int64_t)gi * a.x_group_stride + (int64_t)ri * a.ldx + k0) + col * 16;
    if (i < WCH) wsrc[i] = reinterpret_cast<const char*>(W + (int64_t)(n0 + row) * a.K + k0) + col * 16;
    lds_off[i] = row * TROW + col * 16;
  }
  // two register sets: the global loads of tile kt+2 are in flight while tile kt is
  // multiplied and tile kt+1 (loaded one step earlier) is written to LDS, so each
  // load has a whole k-step of MFMAs to land.  Loads are unconditional (the tail
  // re-reads the last tile) so the compiler's waits stay counted, and the barrier
  // waits for LDS only — __syncthreads() would drain the tile in flight.
  float4_t ra[4 + WCH], rb[4 + WCH];  // [0..3] X chunks, [4..] W chunks
  auto gload = [&](int kt, float4_t* rg) {
    const int kb = kt * TKB;
#pragma unroll
    for (int i = 0; i < 4; ++i) rg[i] = *reinterpret_cast<const float4_t*>(xsrc[i] + kb);
#pragma unroll
    for (int i = 0; i < WCH; ++i) rg[4 + i] = *reinterpret_cast<const float4_t*>(wsrc[i] + kb);
  };
  auto sstore = [&](int buf, const float4_t* rg) {
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<float4_t*>(&smem[buf][lds_off[i]]) = rg[i];
#pragma unroll
    for (int i = 0; i < WCH; ++i) *reinterpret_cast<float4_t*>(&smem[buf][TBM * TROW + lds_off[i]]) = rg[4 + i];
  };
  auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  float4_t acc[4][NI];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = (float4_t){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const char* As = smem[buf];
    const char* Ws = smem[buf] + TBM * TROW;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int koff = (32 * s + 8 * g) * (int)sizeof(T);
      Frag<T> wf[NI], xf[4];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        frag_load(wf[ni], reinterpret_cast<const T*>(Ws + (wc * (TBN_ / 2) + ni * 16 + r) * TROW + koff));
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
        frag_load(xf[mi], reinterpret_cast<const T*>(As + (wr * 64 + mi * 16 + r) * TROW + koff));
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) mfma_step(acc[mi][ni], wf[ni], xf[mi]);
    }
  };

  const int nk = a.K / BK / KZ;
  gload(0, ra);
  gload(min(1, nk - 1), rb);
  sstore(0, ra);
  lds_barrier();
  for (int kt = 0; kt < nk; kt += 2) {
    // LDS buffer 0 holds tile kt, rb holds tile kt+1
    gload(min(kt + 2, nk - 1), ra);
    compute(0);
    if (kt + 1 < nk) sstore(1, rb);
    lds_barrier();
    if (kt + 1 >= nk) break;
    // LDS buffer 1 holds tile kt+1, ra holds tile kt+2
    gload(min(kt + 3, nk - 1), rb);
    compute(1);
    if (kt + 2 < nk) sstore(0, ra);
    lds_barrier();
  }

  if constexpr (KZ > 1) {
    constexpr int NE = 4 * NI;  // float4 per lane of the wave's 64 x TBN_/2 sub-tile
    const int slot = bid * 4 + wave, nslot = ntm * ntn * 4;
    const auto rs = wt_rsrc(a.p1_slab);
    auto off = [&](int z, int e) { return (((z * nslot + slot) * NE + e) * 64 + lane) * 16; };
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) wt_store4(rs, off(kz, mi * NI + ni), acc[mi][ni]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int ticket = 0;
    if (lane == 0) ticket = __hip_atomic_fetch_add(a.p1_cnt + slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ticket = __shfl(ticket, 0, 64);
    if (ticket != KZ - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the add
    if (lane == 0) __hip_atomic_store(a.p1_cnt + slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float4_t pv[4][NI];  // every load issued before the first add
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        pv[mi][ni] = __builtin_bit_cast(float4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, off(1 - kz, mi * NI + ni), 0, 16));
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) acc[mi][ni] += pv[mi][ni];
  }

  // epilogue: lane holds Y[m = m0+wr*64+mi*16+r][n = n0+wc*TBN_/2+ni*16+4g .. +3]
  tile_epilogue<T, EPI, 4, NI, 2>(
      a, acc, [&](int mi) { return m0 + wr * 64 + mi * 16 + r; },
      [&](int ni) { return n0 + wc * (TBN_ / 2) + ni * 16 + 4 * g; });
}

// ============================================================ 256x256 pipelined GEMM (fp16)
// The encoder / cross-KV / conv2 GEMMs (M = 1500 x windows rows, N and K multiples of
// 256 / 128).  Structure (cdna_hip_programming.md §5 "The 256² 8-phase template"):
//   * 8 waves as 2 (M) x 4 (N); a wave owns a 128x64 output tile, acc[8][4] float4;
//   * one K-tile (64) = 4 phases, each computing one 64x32 quadrant of the wave tile
//     (16 MFMAs); phase order Q(0,0) Q(0,1) Q(1,1) Q(1,0), so a phase re-reads only the
//     A or the B half its predecessor did not already hold;
//   * operands reach LDS by global_load_lds (16 B per lane, no VGPR staging) in
//     "stages": half of one operand's tile (128 rows x 64 k = 16 KB = 2 loads per wave),
//     one stage issued per phase, up to 6 stages in flight, retired by ONE counted
//     `s_waitcnt vmcnt` per K-tile — the loads stay in flight across the barriers, which
//     are raw s_barriers (a __syncthreads() would drain them);
//   * the two wave groups (M halves: waves 0-3 and 4-7, one of each per SIMD) run one
//     barrier apart: while one group's MFMAs run, the other issues its LDS reads and
//     stages;
//   * LDS image of a stage: 16 subtiles of 16 rows x 32 k (1 KB), each with the
//     st_16x32 swizzle (16 B chunk index ^= 2 on rows 8-15: conflict-free ds_read_b128),
//     applied on the global SOURCE address of the lane-linear glds write and on the read.
// Stage schedule (phase P = 4t + q of K-tile t, buffer t & 1; stage names SA0 SA1 SB0 SB1
// = A/B halves read in phases {0} {2} {0,3} {1}):
//   q0: SA1(t+1)   q1: SB0(t+1)   q2: SA0(t+2)   q3: SB1(t+2), then vmcnt(4)
// Every stage lands >= 2 phases after the last read of the buffer half it overwrites
// (WAR, both groups), and the vmcnt at q3 retires all of tile t+1 one phase before its
// first read (RAW, a barrier of both groups in between).
namespace g256 {
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int STAGE = 16384;      // one stage: 16 subtiles x 1 KB
constexpr int BUF = 4 * STAGE;    // SA0 SA1 SB0 SB1
enum { SA0 = 0, SA1 = 1, SB0 = 2, SB1 = 3 };
}  // namespace g256

WH_DEV void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}

WH_DEV void glds16(const char* src, char* lds) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src),
                                   (__attribute__((address_space(3))) void*)(lds), 16, 0, 0);
}

// MF = 16: v_mfma_f32_16x16x32_f16 (16 per phase); MF = 32: v_mfma_f32_32x32x16_f16 (8 per
// phase, same operand bytes from the same LDS image: a lane reads row l & 31 of a 32-row
// block, 16 B chunk 2(s & 1) + (l >> 5) of k-step s), acc as 4 x 2 32x32 tiles per wave
template <int EPI, int MF = 16>
__global__ __launch_bounds__(512, 1) void k_gemm_256(GemmArgs a) {
  using namespace g256;
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];  // the kernel's only LDS object

  const int ntn = a.N / BN;
  const int ntm = (a.M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, ntm * ntn);
  const int tm = bid / ntn, tn = bid % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int r = lane & 15, g = lane >> 4;

  // staging: in every stage this wave fills subtiles 2*wave (k 0-31) and 2*wave+1 (k 32-63)
  // of its 16-row block; lane -> row lane>>2, source chunk inverse-swizzled
  const int srow = lane >> 2;
  const int schunk = (lane & 3) ^ ((lane >> 5) << 1);
  const half_t* X = reinterpret_cast<const half_t*>(a.X);
  const half_t* W = reinterpret_cast<const half_t*>(a.W);
  const char* src[4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // SA_h block `wave`: rows wr' * 128 + h * 64 + j * 16 with wr' = wave >> 2, j = wave & 3
    int m = m0 + (wave >> 2) * 128 + h * 64 + (wave & 3) * 16 + srow;
    if (m >= a.M) m = a.M - 1;
    const int gi = m / a.x_group_rows, ri = m - gi * a.x_group_rows;
    src[SA0 + h] = reinterpret_cast<const char*>(X + (int64_t)gi * a.x_group_stride + (int64_t)ri * a.ldx) + schunk * 16;
    // SB_h block `wave`: columns wc' * 64 + h * 32 + j * 16 with wc' = wave >> 1, j = wave & 1
    const int n = n0 + (wave >> 1) * 64 + h * 32 + (wave & 1) * 16 + srow;
    src[SB0 + h] = reinterpret_cast<const char*>(W + (int64_t)n * a.K) + schunk * 16;
  }
  auto stage = [&](int buf, int st, int kt) {
    const char* s = src[st] + kt * (BK * 2);
    char* d = smem + buf * BUF + st * STAGE + wave * 2048;
    glds16(s, d);
    glds16(s + 64, d + 1024);
  };

  // fragment reads: lane (r, g) reads row r, k-chunk g of a subtile, swizzled
  const int roff = r * 64 + ((g ^ ((r >> 3) << 1)) << 4);
  Frag<half_t> af[4][2], bf[2][2];
  auto read_a = [&](int buf, int h) {
    const char* base = smem + buf * BUF + (SA0 + h) * STAGE + wr * 8192 + roff;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) af[mi][ks].v = *reinterpret_cast<const half8_t*>(base + (mi * 2 + ks) * 1024);
  };
  auto read_b = [&](int buf, int h) {
    const char* base = smem + buf * BUF + (SB0 + h) * STAGE + wc * 4096 + roff;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bf[j][ks].v = *reinterpret_cast<const half8_t*>(base + (j * 2 + ks) * 1024);
  };

  // 32x32x16 fragments: X (m) side af32[t][s] for the h-half's two 32-row tiles, W (n)
  // side bf32[s] for the h-half's 32 columns, s = the four 16-deep k-steps of a K-tile
  const int rr = lane & 15, hb = (lane >> 4) & 1, kh = lane >> 5;
  const int coff0 = rr * 64 + (((0 + kh) ^ ((rr >> 3) << 1)) << 4);  // k-steps 0, 2
  const int coff1 = rr * 64 + (((2 + kh) ^ ((rr >> 3) << 1)) << 4);  // k-steps 1, 3
  Frag<half_t> af32[MF == 32 ? 2 : 1][4], bf32[4];
  auto read_a32 = [&](int buf, int h) {
    const char* base = smem + buf * BUF + (SA0 + h) * STAGE + wr * 8192;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int st = 0; st < 4; ++st)
        af32[t][st].v = *reinterpret_cast<const half8_t*>(base + ((t * 2 + hb) * 2 + (st >> 1)) * 1024 +
                                                             ((st & 1) ? coff1 : coff0));
  };
  auto read_b32 = [&](int buf, int h) {
    const char* base = smem + buf * BUF + (SB0 + h) * STAGE + wc * 4096;
#pragma unroll
    for (int st = 0; st < 4; ++st)
      bf32[st].v = *reinterpret_cast<const half8_t*>(base + (hb * 2 + (st >> 1)) * 1024 + ((st & 1) ? coff1 : coff0));
  };
  typedef float f32x16_t __attribute__((ext_vector_type(16)));
  f32x16_t acc32[MF == 32 ? 4 : 1][2];
  float4_t acc[MF == 32 ? 1 : 8][4];
  if constexpr (MF == 32) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc32[i][j] = (f32x16_t){};
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (float4_t){0.f, 0.f, 0.f, 0.f};
  }
  auto rd_a = [&](int buf, int h) {
    if constexpr (MF == 32) read_a32(buf, h);
    else read_a(buf, h);
  };
  auto rd_b = [&](int buf, int h) {
    if constexpr (MF == 32) read_b32(buf, h);
    else read_b(buf, h);
  };

  auto mfma_quadrant = [&](int mh, int nh) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    if constexpr (MF == 32) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int st = 0; st < 4; ++st)
          acc32[mh * 2 + t][nh] =
              __builtin_amdgcn_mfma_f32_32x32x16_f16(bf32[st].v, af32[t][st].v, acc32[mh * 2 + t][nh], 0, 0, 0);
    } else {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) mfma_step(acc[mh * 4 + mi][nh * 2 + j], bf[j][ks], af[mi][ks]);
    }
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = a.K / BK;  // even, >= 2 (launcher)
  // one K-tile from LDS buffer `buf` (compile-time), staging tiles t+1 / t+2
  auto ktile = [&](auto bufc, int t) {
    constexpr int buf = decltype(bufc)::value;
    const bool s1 = t + 1 < nk, s2 = t + 2 < nk;
    // q0: Q(0,0)
    rd_b(buf, 0);
    rd_a(buf, 0);
    if (s1) stage(buf ^ 1, SA1, t + 1);
    raw_barrier();
    mfma_quadrant(0, 0);
    raw_barrier();
    // q1: Q(0,1)
    rd_b(buf, 1);
    if (s1) stage(buf ^ 1, SB0, t + 1);
    raw_barrier();
    mfma_quadrant(0, 1);
    raw_barrier();
    // q2: Q(1,1)
    rd_a(buf, 1);
    if (s2) stage(buf, SA0, t + 2);
    raw_barrier();
    mfma_quadrant(1, 1);
    raw_barrier();
    // q3: Q(1,0); retire tile t+1 before the barrier
    rd_b(buf, 0);
    if (s2) {
      stage(buf, SB1, t + 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    raw_barrier();
    mfma_quadrant(1, 0);
    raw_barrier();
  };

  // prologue: tile 0 complete, SA0 / SB1 of tile 1 in flight
  stage(0, SA0, 0);
  stage(0, SB1, 0);
  stage(0, SA1, 0);
  stage(0, SB0, 0);
  stage(1, SA0, 1);
  stage(1, SB1, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  raw_barrier();
  if (wr == 1) raw_barrier();  // group 1 runs one barrier behind group 0
  for (int t = 0; t < nk; t += 2) {
    ktile(std::integral_constant<int, 0>(), t);
    ktile(std::integral_constant<int, 1>(), t + 1);
  }
  if (wr == 0) raw_barrier();

  if constexpr (MF == 32) {
    // lane holds, per 32x32 tile (mt, nt): m = m0 + wr*128 + mt*32 + (l & 31), n = n0 + wc*64 +
    // nt*32 + 8q + 4(l >> 5) .. +3 in registers 4q .. 4q+3 (q = 0..3)
    float4_t a4[4][8];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int nt = j >> 2, q = j & 3;
        a4[mt][j] = (float4_t){acc32[mt][nt][4 * q], acc32[mt][nt][4 * q + 1], acc32[mt][nt][4 * q + 2],
                               acc32[mt][nt][4 * q + 3]};
      }
    tile_epilogue<half_t, EPI, 4, 8, 2>(
        a, a4, [&](int mt) { return m0 + wr * 128 + mt * 32 + (lane & 31); },
        [&](int j) { return n0 + wc * 64 + (j >> 2) * 32 + 8 * (j & 3) + 4 * kh; });
  } else {
    // lane holds Y[m = m0 + wr*128 + mi*16 + r][n = n0 + wc*64 + ni*16 + 4g .. +3]
    tile_epilogue<half_t, EPI, 8, 4, 4>(
        a, acc, [&](int mi) { return m0 + wr * 128 + mi * 16 + r; },
        [&](int ni) { return n0 + wc * 64 + ni * 16 + 4 * g; });
  }
}

// ============================================================ skinny weight-streaming GEMM
// grid: (ceil(N/16), ceil(M/(16*MT)), ksplit), block 512 = 8 waves.  The block's k-range
// is cut in 32-wide steps dealt round-robin to the 8 waves; per batch of U steps a wave
// issues all its W (HBM) and X (L2) fragment loads before the first MFMA (clamped
// addresses, predicated MFMAs: no branches around loads), then the 8 waves' partial
// tiles are summed in LDS in a fixed order.
template <typename T, int MT, int EPI>
__global__ __launch_bounds__(512) void k_gemv_rows(GemmArgs a) {
  constexpr int NW = 8;
  constexpr int U = sizeof(T) == 2 ? 4 : 2;
  __shared__ float red[NW][MT][64][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int mb = blockIdx.y * (16 * MT);
  const T* X = reinterpret_cast<const T*>(a.X);
  const T* W = reinterpret_cast<const T*>(a.W);

  // split-K: blockIdx.z owns the 32-wide k-steps [S*kz/Z, S*(kz+1)/Z)
  const int kz = blockIdx.z;
  const int S = a.K / 32;
  const int kb = (S * kz / (int)gridDim.z) * 32;
  const int Kc = (S * (kz + 1) / (int)gridDim.z) * 32 - kb;
  int nrow = n0 + r;
  if (nrow >= a.N) nrow = a.N - 1;
  const T* wp = W + (int64_t)nrow * a.K + kb + 8 * g;
  const T* xp[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int m = mb + mt * 16 + r;
    if (m >= a.M) m = a.M - 1;
    const int xr = a.x_rows ? a.x_rows[m] : m;
    xp[mt] = X + (int64_t)xr * a.ldx + kb + 8 * g;
  }
  float4_t acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = (float4_t){0.f, 0.f, 0.f, 0.f};

  const int nsteps = Kc / 32;
  const int last = nsteps - 1;
  for (int b0 = wave; b0 < nsteps; b0 += NW * U) {
    Frag<T> wf[U];
    Frag<T> xf[U][MT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int su = min(b0 + NW * u, last) * 32;
      frag_load(wf[u], wp + su);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) frag_load(xf[u][mt], xp[mt] + su);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (b0 + NW * u < nsteps) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) mfma_step(acc[mt], wf[u], xf[u][mt]);
      }
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
    *reinterpret_cast<float4_t*>(&red[wave][mt][lane][0]) = acc[mt];
  __syncthreads();
  // thread -> (mt, lane) pairs; fixed-order sum over the 8 waves
  for (int idx = tid; idx < MT * 64; idx += 512) {
    const int mt = idx >> 6, ln = idx & 63;
    float4_t v = *reinterpret_cast<float4_t*>(&red[0][mt][ln][0]);
#pragma unroll
    for (int w = 1; w < NW; ++w) v += *reinterpret_cast<float4_t*>(&red[w][mt][ln][0]);
    const int m = mb + mt * 16 + (ln & 15);
    const int n = n0 + 4 * (ln >> 4);
    if (m >= a.M || n >= a.N) continue;
    if (EPI == EPI_F32_COLS) {  // ragged N (vocab): element-wise store
      float* o = a.out_f32 + (int64_t)m * a.ldo;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n + j < a.N) o[n + j] = v[j] + (a.bias ? a.bias[n + j] : 0.f);
      continue;
    }
    if (EPI == EPI_PARTIAL) {
      store4(a.out_f32 + ((int64_t)kz * a.M + m) * a.ldo + n, v[0], v[1], v[2], v[3]);
      continue;
    }
    if (a.bias) v += load4f(a.bias + n);
    epilogue_store<T, EPI>(a, m, 0, m, n, v);
  }
}

// ============================================================ vocabulary projection
// logits[m][n] = sum_k X[m][k] E[n][k] for a decoder step's rows against the whole token
// embedding (V = 51866 columns, 133 MB in fp16).  The rows are cut into a.row_groups groups
// of RG = ceil(M / row_groups) <= 64 rows, each small enough to sit in LDS with all of K
// (fp16, K 1280: <= 60 rows; the launcher uses it for <= 32 rows, one group — two groups
// of 50 at 100 rows measured slower than k_vocab_2p's halves of K); a workgroup stages its group's
// rows once, then every WAVE owns whole 16-column tiles (all of K: no cross-wave reduction,
// no barrier in the loop), visiting tiles gw, gw + nwaves, ... so the weight stream is split
// evenly over the group's waves.  Its weight fragments stream in chunks of VC k-steps, the
// next chunk (of this tile or of the wave's next tile) in flight while the current one is
// multiplied.  The groups of one column range are adjacent logical ids (xcd_remap: one
// XCD), so the second group's weight reads mostly hit that XCD's L2.
// Every output element is one row's dot product in a fixed k order: a row's logits do not
// depend on the other rows or on the grouping (batch invariance).

template <typename T, int MT>
__global__ __launch_bounds__(512) void k_vocab_small(GemmArgs a) {
  constexpr int VC = 8;  // k-steps per chunk
  extern __shared__ __attribute__((aligned(16))) char xsv[];
  const int K = a.K, S = K / 32, nch = (S + VC - 1) / VC;
  const int xrow = K * (int)sizeof(T) + 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  // row group: rows [m0, m0 + RG) of X in LDS rows [0, RG); gridDim.y groups, adjacent ids
  const int ngrp = a.row_groups, RG = (a.M + ngrp - 1) / ngrp;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = lid % ngrp, cblk = lid / ngrp, ncblk = gridDim.x / ngrp;
  const int m0 = grp * RG;
  const T* X = reinterpret_cast<const T*>(a.X);
  const T* W = reinterpret_cast<const T*>(a.W);
  const int nt = (a.N + 15) / 16;
  const int gw = cblk * 8 + wave, nw = ncblk * 8;
  const int ntw = gw < nt ? (nt - 1 - gw) / nw + 1 : 0;  // tiles of this wave
  const int J = ntw * nch;                                 // chunks of this wave
  auto wsrc = [&](int j) {
    const int t = gw + nw * (j / nch), s0 = (j % nch) * VC;
    return W + (int64_t)min(t * 16 + r, a.N - 1) * K + s0 * 32 + 8 * g;
  };
  auto load_chunk = [&](int j, Frag<T>* wf) {
    const T* wp = wsrc(j);
    const int s0 = (j % nch) * VC;
#pragma unroll
    for (int c = 0; c < VC; ++c) frag_load_stream(wf[c], wp + (min(s0 + c, S - 1) - s0) * 32);
  };
  Frag<T> wa[VC], wb[VC];
  float4_t acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = (float4_t){0.f, 0.f, 0.f, 0.f};
  // the first weight chunk is issued before the X staging (it does not depend on X), so its
  // HBM round trip overlaps the LayerNorm prologue's / the X rows' loads
  if (J > 0) load_chunk(0, wa);
  if (a.xf32) {
    // the decoder's final LayerNorm (decoder.py:316) of the fp32 residual rows, recomputed
    // by every workgroup (<= 8 rows x K x 4 B from L2) instead of its own launch: one wave
    // per row, two passes in registers (the arithmetic of k_layernorm / k_proj1)
    constexpr int CPLM = 5;  // float4 chunks per lane: K <= 1280
    const int CH = K / 4;
    for (int row = wave; row < RG; row += 8) {  // M <= 8: one group (launcher)
      T* dst = reinterpret_cast<T*>(xsv + row * xrow);
      if (row >= a.M) {
        for (int c = lane; c < CH; c += 64) store4(dst + 4 * c, 0.f, 0.f, 0.f, 0.f);
        continue;
      }
      const float* xr = a.xf32 + (int64_t)row * K;
      float4_t xv[CPLM], gv[CPLM], bv[CPLM];
#pragma unroll
      for (int i = 0; i < CPLM; ++i) {
        const int c = min(lane + 64 * i, CH - 1);
        xv[i] = load4f(xr + 4 * c);
        gv[i] = load4f(a.ln_g + 4 * c);
        bv[i] = load4f(a.ln_b + 4 * c);
      }
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < CPLM; ++i)
        if (lane + 64 * i < CH) sm += xv[i][0] + xv[i][1] + xv[i][2] + xv[i][3];
      const float mean = wave_sum(sm) / (float)K;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < CPLM; ++i)
        if (lane + 64 * i < CH) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = xv[i][e] - mean;
            q += d * d;
          }
        }
      const float rstd = rsqrtf(wave_sum(q) / (float)K + a.ln_eps);
#pragma unroll
      for (int i = 0; i < CPLM; ++i)
        if (lane + 64 * i < CH) {
          const float4_t v = xv[i];
          store4(dst + 4 * (lane + 64 * i), (v[0] - mean) * rstd * gv[i][0] + bv[i][0],
                 (v[1] - mean) * rstd * gv[i][1] + bv[i][1], (v[2] - mean) * rstd * gv[i][2] + bv[i][2],
                 (v[3] - mean) * rstd * gv[i][3] + bv[i][3]);
        }
    }
  } else {  // stage the group's X rows (rows >= M: zeros)
    // in batches of SB chunks per thread, every load of a batch before its LDS writes
    const int cpr = K * (int)sizeof(T) / 16, total = RG * cpr;
    constexpr int SB = 5;
    for (int c0 = 0; c0 < total; c0 += 512 * SB) {
      float4_t v[SB];
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        const int c = min(c0 + tid + 512 * u, total - 1), row = c / cpr, col = c - row * cpr;
        v[u] = (float4_t){0.f, 0.f, 0.f, 0.f};
        if (m0 + row < a.M) {
          const int xr = a.x_rows ? a.x_rows[m0 + row] : m0 + row;
          v[u] = *reinterpret_cast<const float4_t*>(reinterpret_cast<const char*>(X + (int64_t)xr * a.ldx) + col * 16);
        }
      }
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        const int c = c0 + tid + 512 * u;
        if (c < total) {
          const int row = c / cpr, col = c - row * cpr;
          *reinterpret_cast<float4_t*>(xsv + row * xrow + col * 16) = v[u];
        }
      }
    }
  }
  __syncthreads();
  for (int j = 0; j < J; j += 2) {
    // chunk j in wa (chunk j+1 -> wb in flight), then chunk j+1 in wb (j+2 -> wa)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int jj = j + half;
      if (jj >= J) break;
      Frag<T>* cur = half ? wb : wa;
      Frag<T>* nxt = half ? wa : wb;
      if (jj + 1 < J) load_chunk(jj + 1, nxt);
      const int s0 = (jj % nch) * VC;
#pragma unroll
      for (int c = 0; c < VC; ++c) {
        if (s0 + c < S) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            Frag<T> xf;
            frag_load(xf, reinterpret_cast<const T*>(xsv + min(mt * 16 + r, RG - 1) * xrow) + (s0 + c) * 32 + 8 * g);
            mfma_step(acc[mt], cur[c], xf);
          }
        }
      }
      if (jj % nch == nch - 1) {  // tile done: lane holds rows mt*16 + r, columns n0 + 4g .. +3
        const int n = (gw + nw * (jj / nch)) * 16 + 4 * g;
        // no bias (the launcher requires none): a conditional bias load in the store loop
        // made the compiler wait vmcnt(0) before every store
        const float4_t bv = (float4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int m = m0 + mt * 16 + r;
          if (mt * 16 + r < RG && m < a.M) {
#if WH_WT
            const auto rs = wt_rsrc(a.out_f32);
            if (n + 3 < a.N) {  // one 16-B store (k_vocab_2p's epilogue note)
              wt_store4(rs, (m * a.ldo + n) * 4, acc[mt] + bv);
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (n + e < a.N) wt_store1(rs, (m * a.ldo + n + e) * 4, acc[mt][e] + bv[e]);
            }
#else
            float* o = a.out_f32 + (int64_t)m * a.ldo;
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (n + e < a.N) o[n + e] = acc[mt][e] + bv[e];
#endif
          }
          acc[mt] = (float4_t){0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  }
}

// ============================================================ vocabulary projection, one window
// The single-window step's logits (<= 8 rows: one window's beams, fp16, K = 1280) with the
// decoder's final LayerNorm in the prologue, as k_vocab_small, but balanced over the chip:
// k_vocab_small gives every WAVE whole 16-column tiles over all of K, and 3242 tiles over
// 2048 waves leave 1194 waves with two tiles and 854 with one (the launch lasts two
// tiles: 133 MB at ~4 TB/s).  Here workgroup b owns the contiguous tiles
// [b nt / 256, (b + 1) nt / 256) (12 or 13: every CU streams 520 KB +- 4 %), and its 8 waves
// split K into eighths (5 k-steps each) across ALL of those tiles; the 8 partial tiles are
// summed in LDS in wave order (fixed: deterministic).  The tile loop is unrolled to its
// TMAX = 13 tiles and its weight fragments stream through a ring of D tiles: tile t + D - 1
// is issued while tile t is multiplied, so a wave keeps D x 5 KB in flight from its first
// instruction to its last (a workgroup of 12 tiles re-reads its last tile as the 13th and
// stores nothing for it).  The LayerNorm operands are issued BEFORE the first weight
// fragments, so normalising waits only for them.  Per row the k order is: the wave's 5
// k-steps ascending, the 8 eighths in order — its own fixed order (this kernel serves only
// n_win == 1 batches, whose step is already its own path: DESIGN.md §2).
template <int D>
__global__ __launch_bounds__(512) void k_vocab1(GemmArgs a) {
  CT_MARK(CT_VOCAB, 0);
  constexpr int KW = 8, SW = 5, K = KW * SW * 32, TMAX = 13;  // K 1280, <= 13 tiles (launcher)
  constexpr int XROW = K * 2 + 16;
  extern __shared__ __attribute__((aligned(16))) char xs1[];
  float4_t* red = reinterpret_cast<float4_t*>(xs1 + 8 * XROW);  // [TMAX tiles][KW][64]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int nt = (a.N + 15) / 16, b = blockIdx.x, nb = gridDim.x;
  const int t0 = range_split(b, nt, nb), t1 = range_split(b + 1, nt, nb), ntl = t1 - t0;
  const half_t* W = reinterpret_cast<const half_t*>(a.W);
  const int kb = wave * SW * 32;
  auto load_tile = [&](int tl, Frag<half_t> (&wf)[SW]) {
    const int tile = t0 + min(tl, ntl - 1);
    const half_t* wp = W + (int64_t)min(tile * 16 + r, a.N - 1) * K + kb + 8 * g;
#pragma unroll
    for (int s = 0; s < SW; ++s) frag_load_stream(wf[s], wp + s * 32);
  };
  // the final LayerNorm of the fp32 residual rows (k_vocab_small's prologue): one wave per
  // row; its operands go out first
  constexpr int CPLM = 5;
  const int row = wave;
  const bool lnrow = row < a.M;
  float4_t xv[CPLM], gv[CPLM], bv[CPLM];
  if (lnrow) {
    const float* xr = a.xf32 + (int64_t)row * K;
#pragma unroll
    for (int i = 0; i < CPLM; ++i) {
      const int c = lane + 64 * i;
      xv[i] = load4f(xr + 4 * c);
      gv[i] = load4f(a.ln_g + 4 * c);
      bv[i] = load4f(a.ln_b + 4 * c);
    }
  }
  Frag<half_t> wf[D][SW];
#pragma unroll
  for (int t = 0; t < D - 1; ++t) load_tile(t, wf[t]);
  {
    half_t* dst = reinterpret_cast<half_t*>(xs1 + row * XROW);
    if (!lnrow) {
      for (int c = lane; c < K / 4; c += 64) store4(dst + 4 * c, 0.f, 0.f, 0.f, 0.f);
    } else {
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < CPLM; ++i) sm += xv[i][0] + xv[i][1] + xv[i][2] + xv[i][3];
      const float mean = wave_sum(sm) / (float)K;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < CPLM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = xv[i][e] - mean;
          q += d * d;
        }
      const float rstd = rsqrtf(wave_sum(q) / (float)K + a.ln_eps);
#pragma unroll
      for (int i = 0; i < CPLM; ++i) {
        const float4_t v = xv[i];
        store4(dst + 4 * (lane + 64 * i), (v[0] - mean) * rstd * gv[i][0] + bv[i][0],
               (v[1] - mean) * rstd * gv[i][1] + bv[i][1], (v[2] - mean) * rstd * gv[i][2] + bv[i][2],
               (v[3] - mean) * rstd * gv[i][3] + bv[i][3]);
      }
    }
  }
  __syncthreads();
  // this wave's X fragments (rows r < 8 valid; rows 8..15 repeat row 7, never stored)
  Frag<half_t> xf[SW];
#pragma unroll
  for (int s = 0; s < SW; ++s)
    frag_load(xf[s], reinterpret_cast<const half_t*>(xs1 + min(r, 7) * XROW) + kb + s * 32 + 8 * g);
#pragma unroll
  for (int t = 0; t < TMAX; ++t) {
    if (t + D - 1 < TMAX) load_tile(t + D - 1, wf[(t + D - 1) % D]);
    float4_t acc = (float4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < SW; ++s) mfma_step(acc, wf[t % D][s], xf[s]);
    if (t < ntl) red[(t * KW + wave) * 64 + lane] = acc;
  }
  __syncthreads();
  // per tile: the 8 eighths in wave order; lane (r, g) of a tile: row r, columns 4g .. +3
  const auto rs = wt_rsrc(a.out_f32);
  for (int i = tid; i < ntl * 64; i += 512) {
    const int tl = i >> 6, ln = i & 63, rr = ln & 15, n = (t0 + tl) * 16 + 4 * (ln >> 4);
    float4_t v = red[(tl * KW) * 64 + ln];
#pragma unroll
    for (int w = 1; w < KW; ++w) v += red[(tl * KW + w) * 64 + ln];
    if (rr < a.M) {
      if (n + 3 < a.N) {
        wt_store4(rs, (rr * a.ldo + n) * 4, v);  // one 16-B store (k_vocab_2p's epilogue note): 28.3 -> 27.0 us
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < a.N) wt_store1(rs, (rr * a.ldo + n + e) * 4, v[e]);
      }
    }
  }
  CT_END(CT_VOCAB);
}

// the vocabulary kernels' epilogue: the workgroup's tiles transposed through LDS (the staged
// rows of X are dead), so each store instruction writes 1 KB of one logit row instead of 16
// rows x 64 B (the per-lane form: 7.5 us of k_vocab_2p's epilogue at 100 rows, this ~3)
template <int MT, int NW>
WH_DEV void vocab_store_tr(const GemmArgs& a, const float4_t (&acc)[MT], float* ot, int t0, int t1, bool act, int tid,
                           int wave, int r, int g) {
  constexpr int OTW = NW * 16 + 4;  // floats per staged row (+4: rows 4 banks apart)
  __syncthreads();  // every wave is done with the rows of X
  if (act) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = mt * 16 + r;
      if (m < a.M) *reinterpret_cast<float4_t*>(ot + m * OTW + wave * 16 + 4 * g) = acc[mt];
    }
  }
  __syncthreads();
  const auto rs = wt_rsrc(a.out_f32);
  const int c0 = t0 * 16, nc = min(t1 * 16, a.N) - c0, nc4 = (nc + 3) >> 2;
  for (int i = tid; i < a.M * nc4; i += NW * 64) {
    const int m = i / nc4, c = 4 * (i - m * nc4), n = c0 + c;
    const float4_t v = *reinterpret_cast<const float4_t*>(ot + m * OTW + c);
    if (c + 3 < nc) {
      wt_store4(rs, (m * a.ldo + n) * 4, v);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c + e < nc) wt_store1(rs, (m * a.ldo + n + e) * 4, v[e]);
    }
  }
}

// ============================================================ vocabulary projection, 33-112 rows
// The decoder step's logits for a whole batch (20 windows x 5 beams = 100 rows) against
// the token embedding (133 MB fp16): every row is resident in LDS, HALF of K at a time
// (100 rows x 640 x 2 B = 128 KB), so X crosses L2 once per workgroup and pass (k_gemv_x
// re-stages it per 256-deep subchunk with two barriers each, 85 us; row groups over all of
// K stream every column twice, 89 us: profiles/r03/vocab_groups_ab.txt).  A workgroup of
// 16 waves owns a contiguous range of <= 16 16-column tiles, one per wave; the wave keeps
// its tile's MT accumulators across both passes and streams its weight rows in chunks of
// VC k-steps, the next chunk in flight while one is multiplied.  Accumulation runs over the
// k-steps in ascending order into one accumulator per 16 x 16 block, as in k_vocab_small and
// k_gemv_x: a row's logits are bit-identical whichever kernel the batch size selects.
template <int MT, int DEPTH, bool TR = false>
__global__ __launch_bounds__(1024) void k_vocab_2p(GemmArgs a) {
  CT_MARK(CT_VOCAB, 0);
  constexpr int NW = 16, VC = DEPTH > 2 ? 4 : 5, KH = 640, SH = KH / 32, NCH = SH / VC;  // K 1280 (launcher)
  constexpr int XROW = KH * 2 + 16;
  extern __shared__ __attribute__((aligned(16))) char xs2[];
  constexpr int K = 2 * KH;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int nt = (a.N + 15) / 16;
  const int t0 = range_split(blockIdx.x, nt, gridDim.x), t1 = range_split(blockIdx.x + 1, nt, gridDim.x);
  const int tile = t0 + wave;
  const bool act = tile < t1;
  const half_t* X = reinterpret_cast<const half_t*>(a.X);
  // (the row gather as a wave-uniform pointer test outside the staging: a per-chunk
  // `a.x_rows ? ..` put a vmcnt(0) before every staging load)
  const int* const xrows = a.x_rows;
  const half_t* wrow = reinterpret_cast<const half_t*>(a.W) + (int64_t)min(tile * 16 + r, a.N - 1) * K + 8 * g;
  float4_t acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = (float4_t){0.f, 0.f, 0.f, 0.f};
  // DEPTH weight chunks of VC k-steps: DEPTH - 1 in flight while one is multiplied
  Frag<half_t> wbuf[DEPTH][VC];
  auto load_chunk = [&](int h, int c, Frag<half_t>(&wf)[VC]) {  // k-steps h*SH + c*VC .. +VC-1
    const half_t* wp = wrow + (h * SH + c * VC) * 32;
#pragma unroll
    for (int u = 0; u < VC; ++u) frag_load_stream(wf[u], wp + u * 32);
  };
  constexpr int CPR = KH * 2 / 16;  // 16 B chunks per staged row
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
#ifdef WH_VOCAB_SWAP  // probe build only (the k-step order decides the bits): second half of K
    // first.  The first pass takes ~22 us and the second ~9 whichever half goes first
    // (profiles/r05/vocab_pass_order.txt): an order effect, not a K-half one.  Pass 2's
    // 66 MB in ~9 us (7.5 TB/s) is above any HBM rate measured here — consistent with (not
    // proof of) pass 1 having pulled whole 2560-B rows into the Infinity Cache
    const int h = 1 - hh;
#else
    const int h = hh;
#endif
    // the pass's first DEPTH - 1 weight chunks ride with the staging loads
    if (act) {
#pragma unroll
      for (int c = 0; c < DEPTH - 1 && c < NCH; ++c) load_chunk(h, c, wbuf[c]);
    }
    if (hh) __syncthreads();  // every wave is done with the first half's rows
    if (xrows) {
      for (int c = tid; c < a.M * CPR; c += 1024) {
        const int row = c / CPR, col = c - row * CPR;
        *reinterpret_cast<float4_t*>(xs2 + row * XROW + col * 16) = *reinterpret_cast<const float4_t*>(
            reinterpret_cast<const char*>(X + (int64_t)xrows[row] * a.ldx + h * KH) + col * 16);
      }
    } else {
      // every staging load of the thread issued before the first LDS write (M <= 112: <= 9
      // chunks per thread; the loop form waited a round trip per 16 KB iteration)
      constexpr int SU = (112 * CPR + 1023) / 1024;
      float4_t tmp[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int c = min(tid + 1024 * u, a.M * CPR - 1), row = c / CPR, col = c - row * CPR;
        tmp[u] = *reinterpret_cast<const float4_t*>(reinterpret_cast<const char*>(X + (int64_t)row * a.ldx + h * KH) +
                                                    col * 16);
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int c = tid + 1024 * u;
        if (c < a.M * CPR) {
          const int row = c / CPR, col = c - row * CPR;
          *reinterpret_cast<float4_t*>(xs2 + row * XROW + col * 16) = tmp[u];
        }
      }
    }
    __syncthreads();
    if (hh) CT_MARK(CT_VOCAB, 2);  // the second half of the rows staged
    if (act) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (c + DEPTH - 1 < NCH) load_chunk(h, c + DEPTH - 1, wbuf[(c + DEPTH - 1) % DEPTH]);
#pragma unroll
        for (int u = 0; u < VC; ++u) {
          const int ks = c * VC + u;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            Frag<half_t> xf;
            frag_load(xf, reinterpret_cast<const half_t*>(xs2 + min(mt * 16 + r, a.M - 1) * XROW) + ks * 32 + 8 * g);
            mfma_step(acc[mt], wbuf[c % DEPTH][u], xf);
          }
        }
      }
    }
  }
  CT_MARK(CT_VOCAB, 1);  // the MFMAs issued: the epilogue starts
  if constexpr (TR) {
    vocab_store_tr<MT, NW>(a, acc, reinterpret_cast<float*>(xs2), t0, t1, act, tid, wave, r, g);
    CT_END(CT_VOCAB);
    return;
  }
  if (!act) {
    CT_END(CT_VOCAB);
    return;
  }
  // lane holds rows mt*16 + r, columns tile*16 + 4g .. +3
  const int n = tile * 16 + 4 * g;
  const auto rs = wt_rsrc(a.out_f32);
  // (no bias: the launcher requires none; a conditional bias load here made the compiler
  // wait vmcnt(0) before every store — 28 serialized write-through stores, ~30 of 61 us)
  const float4_t(&ov)[MT] = acc;
  const bool full = n + 3 < a.N;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + r;
    if (m < a.M) {
      if (full) {
        // the lane's 4 columns as ONE 16-B write-through store (whole 64-B row segments per
        // instruction): four 4-B stores per element took the epilogue 15.5 us, this 7.5
        // (k_vocab_2p 49.5 -> 41.6 us at 100 rows, profiles/r05/ab_vocab_wide_stores.txt;
        // rows of the odd-width logit matrix start 8-B aligned: buffer stores take any
        // dword-aligned address)
        wt_store4(rs, (m * a.ldo + n) * 4, ov[mt]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < a.N) wt_store1(rs, (m * a.ldo + n + e) * 4, ov[mt][e]);
      }
    }
  }
  CT_END(CT_VOCAB);
}

// ============================================================ vocabulary projection, one pass over K
// Round 6: k_vocab_2p's tiles, waves and k-step order with ONE pass
// over K.  k_vocab_2p's first pass over K took ~22 us and its second ~9 whichever half went
// first (profiles/r05/vocab_pass_order.txt): the first pulls whole 2560-B embedding rows
// through the memory side and the second re-reads its half from there.  Here each wave
// streams its 16 weight rows front to back once.  LDS holds X k-step-major: slot s =
// [rows][32 halves] (64 B per row, a fragment read is 1 KB contiguous), 24 slots = k-steps
// 0..23 staged up front; k-steps 24..39 refill slots 0..15 once every wave is past k-step
// 15 (their loads issued a chunk earlier, ahead of that chunk's weight loads, so the LDS
// writes wait on nothing the next MFMAs do not), with a second barrier before k-step 24.
// Accumulation order per 16 x 16 block = ascending k-steps, as k_vocab_2p: bit-identical
// logits.  Needs 24 x M x 64 B of LDS (M <= 106).  Measured: no faster than k_vocab_2p
// (the weights stream at ~4.4 TB/s in both, profiles/r06/ab_vocab_1p_kco.txt) — the first
// pass's ~22 us was the HBM stream, not a pass effect; tuning build only (WHISPER_HIP_V1P=1).  GATHER: rows of X named by a.x_rows (a
// template choice: a wave-uniform pointer test per staging load made hipcc wait on each)
constexpr int V1P_SLOTS = 24;
template <int MT, bool GATHER>
__global__ __launch_bounds__(1024) void k_vocab_1p(GemmArgs a) {
  CT_MARK(CT_VOCAB, 0);
  constexpr int NW = 16, VC = 4, DEPTH = 3, K = 1280, S = K / 32, SL = V1P_SLOTS, SR = S - SL, NCH = S / VC;
  static_assert(S % VC == 0 && SR % VC == 0 && SR <= SL, "chunk / slot geometry");
  constexpr int C_FREE = SR / VC;       // first chunk after the refilled slots' last use (k-steps 0..SR-1)
  constexpr int C_REFILL = SL / VC;     // first chunk that reads refilled slots (k-step SL)
  extern __shared__ __attribute__((aligned(16))) char xs1[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
  const int M = a.M, slotB = M * 64;
  const int nt = (a.N + 15) / 16;
  const int t0 = range_split(blockIdx.x, nt, gridDim.x), t1 = range_split(blockIdx.x + 1, nt, gridDim.x);
  const int tile = t0 + wave;
  const bool act = tile < t1;
  const half_t* X = reinterpret_cast<const half_t*>(a.X);
  const int* const xrows = a.x_rows;
  const half_t* wrow = reinterpret_cast<const half_t*>(a.W) + (int64_t)min(tile * 16 + r, a.N - 1) * K + 8 * g;
  float4_t acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = (float4_t){0.f, 0.f, 0.f, 0.f};
  Frag<half_t> wbuf[DEPTH][VC];
  auto load_chunk = [&](int c, Frag<half_t>(&wf)[VC]) {
    const half_t* wp = wrow + c * VC * 32;
#pragma unroll
    for (int u = 0; u < VC; ++u) frag_load_stream(wf[u], wp + u * 32);
  };
  // chunk i of a k-step range: (k-step ks0 + i / (M*4), row, 16-B column) <- X (32-bit
  // buffer offsets: one register per in-flight chunk, not a 64-bit address pair)
  const auto rx = wt_rsrc(X);
  auto src = [&](Frag<half_t>& f, int ks0, int i) {
    const int kk = i / (M * 4), rem = i - kk * M * 4, row = rem >> 2, col = rem & 3;
    const int xr = GATHER ? xrows[row] : row;
    frag_load_buf(f, rx, (xr * a.ldx + (ks0 + kk) * 32 + col * 8) * 2);
  };
  if (act) {
#pragma unroll
    for (int c = 0; c < DEPTH - 1; ++c) load_chunk(c, wbuf[c]);
  }
  {
    constexpr int SU = (106 * SL * 4 + 1023) / 1024;
    const int tot = M * SL * 4;
    Frag<half_t> tmp[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) src(tmp[u], 0, min(tid + 1024 * u, tot - 1));
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int i = tid + 1024 * u;
      if (i < tot) *reinterpret_cast<half8_t*>(xs1 + i * 16) = tmp[u].v;  // slot kk, row, col: i * 16
    }
  }
  __syncthreads();
  // the refill in two parts (the whole refill live across a chunk's MFMAs spilled at MT 7):
  // part j's loads issued at chunk C_FREE - 1 + j ahead of that chunk's weight loads, its LDS
  // writes at chunk C_FREE + j (part 0 after the barrier that frees the slots)
  constexpr int RU = (106 * SR * 4 + 1023) / 1024, RU0 = (RU + 1) / 2;
  static_assert(C_FREE + 1 < C_REFILL, "two refill parts between the barriers");
  const int rtot = M * SR * 4;
  Frag<half_t> rf[RU0];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int u0 = j ? RU0 : 0, u1 = j ? RU : RU0;
      if (c == C_FREE + j) {
        if (j == 0) __syncthreads();  // every wave is past k-step SR - 1: slots 0..SR-1 are free
#pragma unroll
        for (int u = u0; u < u1; ++u) {
          const int i = tid + 1024 * u;
          if (i < rtot) *reinterpret_cast<half8_t*>(xs1 + i * 16) = rf[u - u0].v;
        }
      }
      if (c == C_FREE - 1 + j) {
#pragma unroll
        for (int u = u0; u < u1; ++u) src(rf[u - u0], SL, min(tid + 1024 * u, rtot - 1));
      }
    }
    if (c == C_REFILL) __syncthreads();  // the refilled slots written
    if (act) {
      if (c + DEPTH - 1 < NCH) load_chunk(c + DEPTH - 1, wbuf[(c + DEPTH - 1) % DEPTH]);
#pragma unroll
      for (int u = 0; u < VC; ++u) {
        const int ks = c * VC + u, slot = ks < SL ? ks : ks - SL;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          Frag<half_t> xf;
          frag_load(xf, reinterpret_cast<const half_t*>(xs1 + slot * slotB + min(mt * 16 + r, M - 1) * 64 + 16 * g));
          mfma_step(acc[mt], wbuf[c % DEPTH][u], xf);
        }
      }
    }
  }
  CT_MARK(CT_VOCAB, 1);  // the MFMAs issued: the epilogue starts
  vocab_store_tr<MT, NW>(a, acc, reinterpret_cast<float*>(xs1), t0, t1, act, tid, wave, r, g);
  CT_END(CT_VOCAB);
}

// ============================================================ tall-skinny GEMM, X through LDS
// For 33..128 rows the X operand (L2-resident activations) costs more load bandwidth
// than the weights when every 16-column tile re-reads it.  Here a 256-thread block
// owns 64 columns (one 16-column tile per wave) and stages X[:, k-subchunk] in LDS
// once for its 4 waves; each wave streams its weight rows (all loads of a subchunk in
// flight before the first MFMA).  grid: (ceil(N/64), ceil(M/(16*MT)), ksplit).
constexpr int XS_BYTES = 512;              // bytes of K per LDS subchunk row
constexpr int XS_ROW = XS_BYTES + 16;      // padded row: conflict-free ds_read_b128
template <typename T, int MT, int EPI, int NW = 4>
__global__ __launch_bounds__(64 * NW) void k_gemv_x(GemmArgs a) {
  constexpr int NT = 64 * NW;
  constexpr int KCH = XS_BYTES / (int)sizeof(T);  // k per subchunk (256 half / 128 float)
  constexpr int KS = KCH / 32;                    // k-steps per subchunk
  constexpr int CPR = XS_BYTES / 16;              // 16 B chunks per staged row (32)
  constexpr int NCH = (MT * 16 * CPR + NT - 1) / NT;  // chunks per thread
  constexpr bool RAG = (MT * 16 * CPR) % NT != 0;
  __shared__ __attribute__((aligned(16))) char xs[MT * 16 * XS_ROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16 * NW + wave * 16;
  const int mb = blockIdx.y * (16 * MT);
  const int kz = blockIdx.z;
  const int S = a.K / 32;
  const int kbase = (S * kz / (int)gridDim.z) * 32;
  const int Kc = (S * (kz + 1) / (int)gridDim.z) * 32 - kbase;
  const T* X = reinterpret_cast<const T*>(a.X);
  const T* W = reinterpret_cast<const T*>(a.W);
  int nrow = n0 + r;
  if (nrow >= a.N) nrow = a.N - 1;
  const T* wp = W + (int64_t)nrow * a.K + kbase + 8 * g;
  // this thread's staging chunks: row = c / CPR, 16 B column ch = c % CPR
  const char* xsrc[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = tid + NT * i, row = min(c / CPR, MT * 16 - 1);
    int m = mb + row;
    if (m >= a.M) m = a.M - 1;
    const int xr = a.x_rows ? a.x_rows[m] : m;
    xsrc[i] = reinterpret_cast<const char*>(X + (int64_t)xr * a.ldx + kbase) + (c % CPR) * 16;
  }
  float4_t acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = (float4_t){0.f, 0.f, 0.f, 0.f};
  Frag<T> wf[KS], wn[KS];
  float4_t xr[NCH];
  // issue the loads of subchunk kc (clamped addresses; ragged tails are masked later)
  auto issue = [&](int kc, Frag<T>* w) {
    const int ns = min(KCH, Kc - kc) / 32;
    const int cpr = ns * 2 * (int)sizeof(T);  // valid 16 B chunks per row
#pragma unroll
    for (int s = 0; s < KS; ++s) frag_load_stream(w[s], wp + kc + min(s, ns - 1) * 32);
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int ch = (tid + NT * i) % CPR;
      xr[i] = *reinterpret_cast<const float4_t*>(xsrc[i] + (int64_t)kc * sizeof(T) + (min(ch, cpr - 1) - ch) * 16);
    }
  };
  issue(0, wf);
  for (int kc = 0; kc < Kc; kc += KCH) {
    const int ns = min(KCH, Kc - kc) / 32;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int c = tid + NT * i;
      if (!RAG || c < MT * 16 * CPR) *reinterpret_cast<float4_t*>(xs + (c / CPR) * XS_ROW + (c % CPR) * 16) = xr[i];
    }
    __syncthreads();
    const bool more = kc + KCH < Kc;
    if (more) issue(kc + KCH, wn);  // next subchunk in flight during this one's MFMAs
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s < ns) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          Frag<T> xf;
          frag_load(xf, reinterpret_cast<const T*>(xs + (mt * 16 + r) * XS_ROW) + s * 32 + 8 * g);
          mfma_step(acc[mt], wf[s], xf);
        }
      }
    }
    __syncthreads();
    if (more) {
#pragma unroll
      for (int s = 0; s < KS; ++s) wf[s] = wn[s];
    }
  }
  // lane holds Y[m = mb + mt*16 + r][n = n0 + 4g .. +3]
  const int n = n0 + 4 * g;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mb + mt * 16 + r;
    if (m >= a.M || n >= a.N) continue;
    float4_t v = acc[mt];
    if (EPI == EPI_F32_COLS) {
#if WH_WT
      const auto rs = wt_rsrc(a.out_f32);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n + j < a.N) wt_store1(rs, (m * a.ldo + n + j) * 4, v[j] + (a.bias ? a.bias[n + j] : 0.f));
#else
      float* o = a.out_f32 + (int64_t)m * a.ldo;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n + j < a.N) o[n + j] = v[j] + (a.bias ? a.bias[n + j] : 0.f);
#endif
      continue;
    }
    if (EPI == EPI_PARTIAL) {
#if WH_WT
      wt_store4(wt_rsrc(a.out_f32), (int)((((int64_t)kz * a.M + m) * a.ldo + n) * 4), v);
#else
      store4(a.out_f32 + ((int64_t)kz * a.M + m) * a.ldo + n, v[0], v[1], v[2], v[3]);
#endif
      continue;
    }
    if (a.bias) v += load4f(a.bias + n);
    epilogue_store<T, EPI>(a, m, 0, m, n, v);
  }
}

static int rows_per_block(int M, int mt_block) {
  const int mt = (M + 15) / 16;
  if (mt_block > 0) return std::min(mt_block, std::min(mt, 8));
  return mt >= 8 ? 8 : mt;
}

int gemv_ksplit(int M, int N, int K, int max_z, int mt_block) {
  // split-K for the skinny paths.  One block's latency is nearly independent of its
  // k-range at these sizes, so the wall time is one block's latency as long as the
  // blocks fit on the CUs at once: take the largest z with blocks <= the target
  // (default 256 = one per CU; WHISPER_HIP_GEMV_WGS overrides for tuning).
  const char* env = tune_env("WHISPER_HIP_GEMV_WGS");
  const int target = env ? atoi(env) : 256;
  const int mt = (M + 15) / 16;
  const bool xpath = mt >= 3;  // k_gemv_x (EPI_PARTIAL with >= 33 rows)
  const int rp = rows_per_block(M, mt_block);
  const int wgs = (xpath ? (N + 63) / 64 : (N + 15) / 16) * ((M + 16 * rp - 1) / (16 * rp));
  const int steps = K / 32;
  int best = 1;
  for (int z = 1; z <= 16 && z <= max_z && z <= steps; ++z)
    if (wgs * z <= target) best = z;
  return best;
}

// ============================================================ launchers
template <typename T>
int launch_gemm_tiles(const GemmArgs& a, int epi, int tile_sel, hipStream_t st);

template <typename T>
int launch_gemm(const GemmArgs& a, int epi, hipStream_t st) {
  static const int tile_sel = [] {  // WHISPER_HIP_GEMM=128 keeps the 128x128 kernel (A/B)
    const char* e = tune_env("WHISPER_HIP_GEMM");
    return e ? atoi(e) : 256;
  }();
  return launch_gemm_tiles<T>(a, epi, tile_sel, st);
}

template <typename T>
int launch_gemm_tiles(const GemmArgs& a, int epi, int tile_sel, hipStream_t st) {
  if (a.M <= 0) return 0;
  const bool big = a.M > 128 && (a.N % TBN) == 0 && (a.K % (TKB / (int)sizeof(T))) == 0 && epi != EPI_F32_COLS &&
                   epi != EPI_PARTIAL && a.x_rows == nullptr;
  const bool t256 = big && sizeof(T) == 2 && (tile_sel == 256 || tile_sel == 257) && a.M >= 256 && (a.N % g256::BN) == 0 &&
                    (a.K % (2 * g256::BK)) == 0 && epi != EPI_QKV_DEC &&
                    // below one 256-tile per CU the 128-tile grid fills the chip better
                    // (tools/gemm_bench: one window, fc1: 0.035 vs 0.039 ms)
                    ((a.M + g256::BM - 1) / g256::BM) * (a.N / g256::BN) >= 256;
  if (t256) {
    const int nwg = ((a.M + g256::BM - 1) / g256::BM) * (a.N / g256::BN);
    switch (epi) {
#define CASE(E)                                                   \
  case E:                                                         \
    if (tile_sel == 257) k_gemm_256<E, 32><<<nwg, 512, 0, st>>>(a), wh_launched("k_gemm_256"); \
    else k_gemm_256<E><<<nwg, 512, 0, st>>>(a), wh_launched("k_gemm_256");                    \
    break;
      CASE(EPI_STORE) CASE(EPI_STORE_GELU) CASE(EPI_RESID) CASE(EPI_GELU_POS) CASE(EPI_HEADSPLIT) CASE(EPI_QKV_ENC)
#undef CASE
      default: return -1;
    }
  } else if (big) {
    const int ntm = (a.M + TBM - 1) / TBM;
    // under one 128 x 128 tile per CU, 128 x 64 tiles double the grid (a single window's
    // n-wide encoder GEMMs: 120 -> 240 workgroups)
    const bool half = ntm * (a.N / TBN) < 256 && (a.N % 64) == 0 && tile_sel != 129;
    const int nwg = ntm * (a.N / (half ? 64 : TBN));
    // two K halves per 128 x 64 tile where the caller hands over slabs + counters (the
    // single-window encoder's residual GEMMs: out, fc2, conv2); p1_slabs in KB, 64 per tile
    const bool kz2 = half && sizeof(T) == 2 && (epi == EPI_RESID || epi == EPI_GELU_POS) && a.p1_slab && a.p1_cnt &&
                     (a.K / (TKB / (int)sizeof(T))) % 2 == 0 && (int64_t)nwg * 64 <= a.p1_slabs && tile_sel != 128;
    if (kz2) {
      if (epi == EPI_RESID) k_gemm_tile<T, EPI_RESID, 64, 2><<<2 * nwg, 256, 0, st>>>(a), wh_launched("k_gemm_tile");
      else k_gemm_tile<T, EPI_GELU_POS, 64, 2><<<2 * nwg, 256, 0, st>>>(a), wh_launched("k_gemm_tile");
      return 0;
    }
    switch (epi) {
#define CASE(E)                                                       \
  case E:                                                             \
    if (half) k_gemm_tile<T, E, 64><<<nwg, 256, 0, st>>>(a), wh_launched("k_gemm_tile");          \
    else k_gemm_tile<T, E><<<nwg, 256, 0, st>>>(a), wh_launched("k_gemm_tile");                   \
    break;
      CASE(EPI_STORE) CASE(EPI_STORE_GELU) CASE(EPI_RESID) CASE(EPI_GELU_POS) CASE(EPI_HEADSPLIT) CASE(EPI_QKV_DEC)
      CASE(EPI_QKV_ENC)
#undef CASE
      default: return -1;
    }
  } else {
    if (a.K % 32) return -2;
    if (a.x_group_rows != a.M && a.x_group_rows != 0 && a.x_group_rows < a.M) return -3;  // skinny: plain rows only
    const int mt = (a.M + 15) / 16;
    const int rows_per = rows_per_block(a.M, a.mt_block);
    const int ks = epi == EPI_PARTIAL ? a.ksplit : 1;
    if (ks < 1 || ks > a.K / 32) return -4;
    static const bool vocab_small = [] {  // WHISPER_HIP_VOCAB_SMALL=0: the k_gemv path (A/B)
      const char* e = tune_env("WHISPER_HIP_VOCAB_SMALL");
      return !(e && e[0] == '0');
    }();
    if (a.xf32 && !(vocab_small && epi == EPI_F32_COLS && a.N >= 16384 && a.M <= 8 && a.K <= 1280 && a.K % 32 == 0 &&
                    !a.x_rows))
      return -6;  // the LayerNorm prologue exists only in k_vocab_small / k_vocab1
    // the single-window step (LayerNorm prologue, fp16, K 1280): k_vocab1, balanced over the
    // chip (WHISPER_HIP_VOCAB1=0 in the tuning build: k_vocab_small)
    static const bool vocab1 = [] {
      const char* e = tune_env("WHISPER_HIP_VOCAB1");
      return !(e && e[0] == '0');
    }();
    if (sizeof(T) == 2 && vocab1 && a.xf32 && a.K == 1280 && !a.bias && a.M <= 8 && (a.N + 15) / 16 <= 256 * 13) {
      constexpr int D = 6;  // (N + 15) / 16 <= 256 x 13: at most 13 tiles per workgroup (TMAX)
      const int lds = 8 * (1280 * 2 + 16) + 13 * 8 * 64 * 16;
      static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vocab1<D>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
      if (!attr) return -5;
      k_vocab1<D><<<256, 512, lds, st>>>(a), wh_launched("k_vocab1");
      return 0;
    }
    // k_vocab_small: the rows in groups of <= 64 that fit LDS with all of K (152 KB)
    const int vxrow = a.K * (int)sizeof(T) + 16;
    const int vrg_max = std::min(64, (152 * 1024) / vxrow);
    const int vgrp = (a.M + vrg_max - 1) / vrg_max;
    // (<= 32 rows: at 100 rows, 2 groups of 50, it measured 89.2 us against k_gemv_x's 84.6:
    // each CU streams its column block twice, profiles/r03/vocab_groups_ab.txt)
    if (vocab_small && epi == EPI_F32_COLS && !a.bias && a.N >= 16384 && a.M <= (sizeof(T) == 2 ? 32 : 16) && vgrp <= 4 &&
        a.K <= 1280 && a.K % 32 == 0) {
      const int rg = (a.M + vgrp - 1) / vgrp, mtv = (rg + 15) / 16;
      const int lds = rg * vxrow;
      const int grid = vgrp * std::max(1, std::min(256 / vgrp, (a.N + 127) / 128));
      GemmArgs av = a;
      av.row_groups = vgrp;
      auto go = [&](auto mtc) {  // one attribute flag per instantiation
        constexpr int MTV = decltype(mtc)::value;
        static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vocab_small<T, MTV>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
        if (!attr) return -5;
        k_vocab_small<T, MTV><<<grid, 512, lds, st>>>(av), wh_launched("k_vocab_small");
        return 0;
      };
      switch (mtv) {
        case 1: return go(std::integral_constant<int, 1>());
        case 2: return go(std::integral_constant<int, 2>());
        case 3: return go(std::integral_constant<int, 3>());
        default: return go(std::integral_constant<int, 4>());
      }
    }
    // k_vocab_2p: 33..112 fp16 rows resident in LDS, half of K per pass
    if (sizeof(T) == 2 && vocab_small && epi == EPI_F32_COLS && !a.bias && a.N >= 16384 && a.M > 32 && a.M <= 112 &&
        !a.xf32 &&
        a.K == 1280 && a.M * (a.K + 16) <= 150 * 1024) {
      // two 4-step weight chunks in flight per wave (DEPTH 3; WHISPER_HIP_V2P_DEPTH=2 in the
      // tuning build: one 5-step chunk) — step graph 3.5456 -> 3.5413 ms at 20 windows,
      // profiles/r03/step_tail_ab.txt
      const char* de = tune_env("WHISPER_HIP_V2P_DEPTH");
      const bool d3 = !(de && de[0] == '2');
      // the epilogue through LDS, one 1-KB row segment per store instruction: 41.7 / 42.0 ->
      // 37.4 / 37.4 us at 100 rows, step graph 3.244 / 3.251 -> 3.237 / 3.238 ms
      // (profiles/r05/ab_vocab_epilogue_lds.txt).  Tuning: WHISPER_HIP_V2P_TR=0 -> per lane
      const char* te = tune_env("WHISPER_HIP_V2P_TR");
      const bool tr = !(te && te[0] == '0');
      const int nt = (a.N + 15) / 16;
      const int grid = std::max((nt + 15) / 16, std::min(256, nt));
      const int lds = a.M * (a.K + 16);  // rows x (K / 2 halves x 2 B + 16)
      // tuning build, WHISPER_HIP_V1P=1: k_vocab_1p (one pass over K) when its 24 k-step
      // slots fit (M <= 106).  Measured equal: weights-in to epilogue start ~30 us either way
      // (20 windows: step 3.186 / 3.187 ms at 12 tokens, profiles/r06/ab_vocab_1p_kco.txt)
      const char* v1e = tune_env("WHISPER_HIP_V1P");
      const bool v1p = v1e && v1e[0] == '1' && tr && V1P_SLOTS * a.M * 64 <= 160 * 1024;
      auto go = [&](auto mtc) {
        constexpr int MTV = decltype(mtc)::value;
        if (v1p) {
          const int lds1 = std::max(V1P_SLOTS * a.M * 64, a.M * (16 * 16 + 4) * 4);
          static bool attr1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vocab_1p<MTV, true>),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess &&
                              hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vocab_1p<MTV, false>),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
          if (!attr1) return -5;
          if (a.x_rows) k_vocab_1p<MTV, true><<<grid, 1024, lds1, st>>>(a), wh_launched("k_vocab_1p");
          else k_vocab_1p<MTV, false><<<grid, 1024, lds1, st>>>(a), wh_launched("k_vocab_1p");
          return 0;
        }
        static bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vocab_2p<MTV, 2>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess &&
                           hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vocab_2p<MTV, 3>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
        if (!attr) return -5;
        if (tr) {  // the LDS-transposed epilogue (needs the staged rows' LDS: M x 1 KB + pad)
          static bool attr_t = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vocab_2p<MTV, 3, true>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
          if (!attr_t) return -5;
          k_vocab_2p<MTV, 3, true><<<grid, 1024, std::max(lds, a.M * (16 * 16 + 4) * 4), st>>>(a), wh_launched("k_vocab_2p");
          return 0;
        }
        if (d3) k_vocab_2p<MTV, 3><<<grid, 1024, lds, st>>>(a), wh_launched("k_vocab_2p");
        else k_vocab_2p<MTV, 2><<<grid, 1024, lds, st>>>(a), wh_launched("k_vocab_2p");
        return 0;
      };
      switch ((a.M + 15) / 16) {
        case 3: return go(std::integral_constant<int, 3>());
        case 4: return go(std::integral_constant<int, 4>());
        case 5: return go(std::integral_constant<int, 5>());
        case 6: return go(std::integral_constant<int, 6>());
        default: return go(std::integral_constant<int, 7>());
      }
    }
    if (mt >= 3 && epi == EPI_F32_COLS && a.N >= 16384) {
      // vocabulary projection: NW column tiles share each staged X subchunk, so X
      // (re-read from L2 by every workgroup) costs 112/(16 NW) of the weight bytes
      static const int nw = [] {
        const char* e = tune_env("WHISPER_HIP_VOCAB_WAVES");
        const int v = e ? atoi(e) : 8;
        return v == 4 ? 4 : 8;  // 16 waves spill
      }();
      dim3 gv((a.N + 16 * nw - 1) / (16 * nw), (a.M + 16 * rows_per - 1) / (16 * rows_per), 1);
#define LAUNCHV(MT_)                                                                                  \
  switch (nw) {                                                                                      \
    case 4: k_gemv_x<T, MT_, EPI_F32_COLS, 4><<<gv, 256, 0, st>>>(a), wh_launched("k_gemv_x"); break;                         \
    default: k_gemv_x<T, MT_, EPI_F32_COLS, 8><<<gv, 512, 0, st>>>(a), wh_launched("k_gemv_x"); break;                        \
  }
      switch (rows_per) {
        case 3: LAUNCHV(3) break;
        case 4: LAUNCHV(4) break;
        case 5: LAUNCHV(5) break;
        case 6: LAUNCHV(6) break;
        case 7: LAUNCHV(7) break;
        default: LAUNCHV(8) break;
      }
#undef LAUNCHV
      return 0;
    }
    // tall-skinny split-K partials: X shared via LDS by 4 column tiles.  Every other
    // epilogue at <= 128 rows runs k_gemv_rows below whatever the row count, so a row's
    // summation order (8 waves' k-step shares, summed in fixed order) does not depend on
    // how many rows share the launch — the first pass of a batch of windows is
    // batch-invariant like the step (fc1 used to switch to k_gemv_x from 33 rows)
    if (mt >= 3 && epi == EPI_PARTIAL) {
      dim3 gx((a.N + 63) / 64, (a.M + 16 * rows_per - 1) / (16 * rows_per), ks);
#define LAUNCHX(MT_)                                                                            \
  switch (epi) {                                                                               \
    case EPI_STORE: k_gemv_x<T, MT_, EPI_STORE><<<gx, 256, 0, st>>>(a), wh_launched("k_gemv_x"); break;                  \
    case EPI_STORE_GELU: k_gemv_x<T, MT_, EPI_STORE_GELU><<<gx, 256, 0, st>>>(a), wh_launched("k_gemv_x"); break;        \
    case EPI_RESID: k_gemv_x<T, MT_, EPI_RESID><<<gx, 256, 0, st>>>(a), wh_launched("k_gemv_x"); break;                  \
    case EPI_QKV_DEC: k_gemv_x<T, MT_, EPI_QKV_DEC><<<gx, 256, 0, st>>>(a), wh_launched("k_gemv_x"); break;              \
    case EPI_F32_COLS: k_gemv_x<T, MT_, EPI_F32_COLS><<<gx, 256, 0, st>>>(a), wh_launched("k_gemv_x"); break;            \
    case EPI_PARTIAL: k_gemv_x<T, MT_, EPI_PARTIAL><<<gx, 256, 0, st>>>(a), wh_launched("k_gemv_x"); break;              \
    default: return -1;                                                                        \
  }
      switch (rows_per) {
        case 3: LAUNCHX(3) break;
        case 4: LAUNCHX(4) break;
        case 5: LAUNCHX(5) break;
        case 6: LAUNCHX(6) break;
        case 7: LAUNCHX(7) break;
        default: LAUNCHX(8) break;
      }
#undef LAUNCHX
      return 0;
    }
    dim3 grid((a.N + 15) / 16, (a.M + 16 * rows_per - 1) / (16 * rows_per), ks);
#define LAUNCH(MT_)                                                                             \
  switch (epi) {                                                                               \
    case EPI_STORE: k_gemv_rows<T, MT_, EPI_STORE><<<grid, 512, 0, st>>>(a), wh_launched("k_gemv_rows"); break;             \
    case EPI_STORE_GELU: k_gemv_rows<T, MT_, EPI_STORE_GELU><<<grid, 512, 0, st>>>(a), wh_launched("k_gemv_rows"); break;   \
    case EPI_RESID: k_gemv_rows<T, MT_, EPI_RESID><<<grid, 512, 0, st>>>(a), wh_launched("k_gemv_rows"); break;             \
    case EPI_HEADSPLIT: k_gemv_rows<T, MT_, EPI_HEADSPLIT><<<grid, 512, 0, st>>>(a), wh_launched("k_gemv_rows"); break;     \
    case EPI_QKV_DEC: k_gemv_rows<T, MT_, EPI_QKV_DEC><<<grid, 512, 0, st>>>(a), wh_launched("k_gemv_rows"); break;         \
    case EPI_F32_COLS: k_gemv_rows<T, MT_, EPI_F32_COLS><<<grid, 512, 0, st>>>(a), wh_launched("k_gemv_rows"); break;       \
    case EPI_PARTIAL: k_gemv_rows<T, MT_, EPI_PARTIAL><<<grid, 512, 0, st>>>(a), wh_launched("k_gemv_rows"); break;         \
    default: return -1;                                                                        \
  }
    switch (rows_per) {
      case 1: LAUNCH(1) break;
      case 2: LAUNCH(2) break;
      case 3: LAUNCH(3) break;
      case 4: LAUNCH(4) break;
      case 5: LAUNCH(5) break;
      case 6: LAUNCH(6) break;
      case 7: LAUNCH(7) break;
      default: LAUNCH(8) break;
    }
#undef LAUNCH
  }
  return 0;
}

template int launch_gemm<float>(const GemmArgs&, int, hipStream_t);
template int launch_gemm_tiles<half_t>(const GemmArgs&, int, int, hipStream_t);
template int launch_gemm<half_t>(const GemmArgs&, int, hipStream_t);

}  // namespace wh

#if WH_TUNING
WH_CT_READER(gemm)
#endif
