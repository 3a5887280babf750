// Launcher for k_proj (wh_proj.h): the split-K projections of the decoder step.
//
// Output format is the k_gemv_x EPI_PARTIAL one (fp32 slabs out_f32[z][M][N]), so the
// consumers (k_resid_ln, k_reduce_store, k_self_attn_qkv) are unchanged.  The tile
// configuration is picked per shape from a short list: rows in one row group when
// M <= 112 (MT = ceil(M/16)), then — among tiles of at least 5 k-steps per wave — the
// configuration with the most workgroups that still fits one workgroup per CU (256).
// Measured on MI355X at 100 rows (tools/proj_bench.hip, profiles/r01/proj_bench.txt):
// qkv 4.0, out 6.0, fc1 / fc2 11.2 -> 8.3 us per launch against k_gemv_x; in the
// large-v3 beam step, 1280 x 1280 at 8 slabs (160 workgroups) instead of 4-step tiles
// at 10 slabs (200) took the step from 4.20 to 3.97 ms (WHISPER_HIP_PROJ_FORCE sweep,
// profiles/r01/proj_force_sweep.txt).
#include <array>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "wh_proj.h"
#include <hip/hip_ext.h>

namespace wh {

namespace {

struct Cfg { int nsub, kw, nstep; };
constexpr Cfg CFGS[] = {{4, 1, 5}, {4, 1, 10}, {5, 1, 10}, {4, 1, 4}, {4, 1, 6},
                        {4, 1, 20}, {5, 1, 20}, {8, 1, 5}, {8, 1, 10}};
constexpr int NCFG = sizeof(CFGS) / sizeof(CFGS[0]);

typedef void (*KFn)(GemmArgs);
struct Ent { KFn f; int lds; };

template <typename T, int MT, int C>
Ent ent() {
  constexpr Cfg c = CFGS[C];
  return {&k_proj<T, MT, c.nsub, c.kw, c.nstep, EPI_PARTIAL>, ProjShape<T, MT, c.nsub, c.kw, c.nstep>::LDS};
}
template <typename T, int MT>
void row(Ent* e) {
  e[0] = ent<T, MT, 0>(); e[1] = ent<T, MT, 1>(); e[2] = ent<T, MT, 2>(); e[3] = ent<T, MT, 3>(); e[4] = ent<T, MT, 4>();
  e[5] = ent<T, MT, 5>(); e[6] = ent<T, MT, 6>(); e[7] = ent<T, MT, 7>(); e[8] = ent<T, MT, 8>();
}
template <typename T>
struct Table {
  Ent e[7][NCFG];
  bool attr[7][NCFG] = {};
  Table() {
    row<T, 1>(e[0]); row<T, 2>(e[1]); row<T, 3>(e[2]); row<T, 4>(e[3]);
    row<T, 5>(e[4]); row<T, 6>(e[5]); row<T, 7>(e[6]);
  }
};

constexpr int LDS_MAX = 160 * 1024;

}  // namespace

template <typename T>
int launch_proj_partial(const GemmArgs& a, int max_z, hipStream_t st, int* z_out, hipEvent_t ev0, hipEvent_t ev1) {
  static Table<T> tab;
  static const bool off = [] {
    const char* e = tune_env("WHISPER_HIP_PROJ");
    return e && e[0] == '0';
  }();
  if (off || a.M < 1 || a.M > 112 || a.K % 32 || a.N % 16 || a.x_group_rows < a.M) return -1;
  const int mt = (a.M + 15) / 16, S = a.K / 32;
  // tuning override: WHISPER_HIP_PROJ_FORCE="N:K:cfg,..." pins the CFGS entry per shape
  static const std::vector<std::array<int, 3>> force = [] {
    std::vector<std::array<int, 3>> v;
    if (const char* e = tune_env("WHISPER_HIP_PROJ_FORCE")) {
      int n, k, c, off = 0, used = 0;
      while (sscanf(e + off, "%d:%d:%d%n", &n, &k, &c, &used) == 3) {
        v.push_back({n, k, c});
        off += used;
        if (e[off] == ',') ++off;
        else break;
      }
    }
    return v;
  }();
  int forced = -1;
  for (const auto& f : force)
    if (f[0] == a.N && f[1] == a.K && f[2] >= 0 && f[2] < NCFG) forced = f[2];
  int best = -1, best_wgs = 0, best_z = 0;
  for (int c = 0; c < NCFG; ++c) {
    const Cfg& k = CFGS[c];
    if (S % (k.kw * k.nstep)) continue;
    const int z = S / (k.kw * k.nstep);
    // feasibility at the largest row tile count (MT 7): a configuration whose LDS fits
    // only at fewer rows would give small batches another K split (and so other slab
    // sums) than large ones — caught by test_gpu_batch.py::test_batch_invariance_fp16
    if (z > 16 || tab.e[6][c].lds > LDS_MAX) continue;
    const int wgs = (a.N + 16 * k.nsub - 1) / (16 * k.nsub) * z;
    if (forced >= 0) {
      if (c == forced) best = c, best_wgs = wgs, best_z = z;
      continue;
    }
    if (wgs > 256) continue;
    // rank: at least 5 k-steps per wave first (4-step tiles measured 7.8 us against
    // 5-step tiles' 5.x us in the large-v3 step: 10 slabs instead of 8 and a
    // latency-bound wave), then the most workgroups, then the longer k-range
    const bool deep = k.nstep >= 5;
    const bool bdeep = best >= 0 && CFGS[best].nstep >= 5;
    if (best < 0 || (deep && !bdeep) ||
        (deep == bdeep && (wgs > best_wgs || (wgs == best_wgs && k.nstep > CFGS[best].nstep))))
      best = c, best_wgs = wgs, best_z = z;
  }
  // the tiling (and so every row's summation order) is chosen from the weight shape
  // alone, never from the row count: a window's step is batch-invariant.
  // max_z is only the slab capacity the caller has for this row count
  if (best < 0 || best_z > max_z) return -1;
  const Ent& e = tab.e[mt - 1][best];
  if (!tab.attr[mt - 1][best]) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(e.f), hipFuncAttributeMaxDynamicSharedMemorySize, e.lds) !=
        hipSuccess)
      return -2;
    tab.attr[mt - 1][best] = true;
  }
  GemmArgs b = a;
  b.ksplit = best_z;
  if (ev0)
    hipExtLaunchKernelGGL(e.f, dim3(best_wgs), dim3(64 * CFGS[best].nsub * CFGS[best].kw), e.lds, st, ev0, ev1, 0, b), wh_launched("k_proj");
  else {
    hipLaunchKernelGGL(e.f, dim3(best_wgs), dim3(64 * CFGS[best].nsub * CFGS[best].kw), e.lds, st, b);
    wh_launched("k_proj");
  }
  *z_out = best_z;
  return 0;
}

// ------------------------------------------------------------ k_proj1 (single-window step)
// Configurations per model width n (S = n / 32 k-steps = BKW x NS), (nsub, kw, nstep, zs):
//   qkv (n -> 3n) and cross-q (n -> n), LayerNorm prologue: (1, BKW, NS, 1), whole K;
//   fc1 (n -> 4n), LayerNorm prologue: (F1SUB, BKW, NS, 1), whole K (32 columns per
//     workgroup at n = 1280 in fp16: 160 workgroups; fp32 keeps 16, its 16-wave form spills);
//   out, cross-out (n -> n, residual): (1, BKW / 2, NS, 2);  fc2 (4n -> n): (1, 2 BKW, NS, 2).
// Measured at n = 1280 (large-v3, 5 rows, graph-mode rocprof, profiles/r02/p1_tilings.txt):
// the in-launch reduction's cost grows with the split count — k_proj's own tilings with
// 4-16 slices per tile took 6.6 / 10.3 / 9.3 / 8.1 / 7.5 us (nn / fc2 / fc1 / cross-q / qkv)
// against 5.5 / 8.0 / 8.3 / 5.4 / 5.7 us for the tilings here, which split only the
// residual projections, in two.
namespace {
template <typename T, int NSUB, int KW, int NS, int ZS, int CPL, int EPI, int MODE = 0>
int p1_go(const GemmArgs& a, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
  using P = Proj1Shape<T, NSUB, KW, NS, CPL>;
  static_assert(P::LDS <= 64 * 1024, "k_proj1 LDS");
  static_assert(NSUB * KW <= 16, "k_proj1 waves");
  if (a.K != ZS * P::KC || a.N % (16 * NSUB)) return -1;
  if (ZS > 1 && (!a.p1_slab || !a.p1_cnt || (int64_t)ZS * (a.N / 16) > a.p1_slabs)) return -1;
  if ((MODE & P1_PEND) && (!a.res_slab || !a.res_bias || !a.x_out || a.x_out == a.xf32)) return -1;
  const dim3 grid(a.N / (16 * NSUB), ZS), block(64 * NSUB * KW);
  void (*f)(GemmArgs) = &k_proj1<T, NSUB, KW, NS, ZS, CPL, EPI, MODE>;
  if (ev0)
    hipExtLaunchKernelGGL(f, grid, block, P::LDS, st, ev0, ev1, 0, a), wh_launched("k_proj1");
  else {
    hipLaunchKernelGGL(f, grid, block, P::LDS, st, a);
    wh_launched("k_proj1");
  }
  return 0;
}

// one model width: the five kernels its step uses
template <typename T, int CPL, int BKW, int NS, int F1SUB>
int p1_width_launch(const GemmArgs& a, int epi, bool ln, int n, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  if (ln) {
    if (a.K != n) return -1;
    if (a.res_slab) {  // a deferred residual is pending on the input rows
      if (epi == EPI_QKV_DEC && a.N == 3 * n) return p1_go<T, 1, BKW, NS, 1, CPL, EPI_QKV_DEC, P1_PEND>(a, st, e0, e1);
      if (epi == EPI_STORE_GELU && a.N == 4 * n)
        return p1_go<T, F1SUB, BKW, NS, 1, CPL, EPI_STORE_GELU, P1_PEND>(a, st, e0, e1);
      if (epi == EPI_STORE && a.N == n) return p1_go<T, 1, BKW, NS, 1, CPL, EPI_STORE, P1_PEND>(a, st, e0, e1);
      return -1;
    }
    if (epi == EPI_QKV_DEC && a.N == 3 * n) return p1_go<T, 1, BKW, NS, 1, CPL, EPI_QKV_DEC>(a, st, e0, e1);
    if (epi == EPI_STORE_GELU && a.N == 4 * n) return p1_go<T, F1SUB, BKW, NS, 1, CPL, EPI_STORE_GELU>(a, st, e0, e1);
    if (epi == EPI_STORE && a.N == n) return p1_go<T, 1, BKW, NS, 1, CPL, EPI_STORE>(a, st, e0, e1);
    return -1;
  }
  if (epi != EPI_RESID || a.N != n) return -1;
  if (a.p1_defer) {
    if (a.K == n) return p1_go<T, 1, BKW / 2, NS, 2, 0, EPI_RESID, P1_DEFER>(a, st, e0, e1);
    if (a.K == 4 * n) return p1_go<T, 1, 2 * BKW, NS, 2, 0, EPI_RESID, P1_DEFER>(a, st, e0, e1);
    return -1;
  }
  if (a.K == n) return p1_go<T, 1, BKW / 2, NS, 2, 0, EPI_RESID>(a, st, e0, e1);
  if (a.K == 4 * n) return p1_go<T, 1, 2 * BKW, NS, 2, 0, EPI_RESID>(a, st, e0, e1);
  return -1;
}
}  // namespace

bool proj1_supported(int R, int n) {
  if (R < 1 || R > P1_RMAX) return false;
  switch (n) {
    case 1280: case 1024: case 768: case 512: case 384: case 128: return true;
    default: return false;
  }
}

template <typename T>
int launch_proj1(const GemmArgs& a, int epi, bool ln, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
  if (a.M < 1 || a.M > P1_RMAX || a.N % 16 || !a.bias) return -1;
  if (ln && (!a.xf32 || !a.ln_g || !a.ln_b)) return -1;
  // the model width: the LayerNorm'd input (K) or the residual output (N)
  const int n = ln ? a.K : a.N;
  switch (n) {  //                            CPL BKW NS F1SUB
    case 1280: return p1_width_launch<T, 5, 8, 5, sizeof(T) == 2 ? 2 : 1>(a, epi, ln, n, st, ev0, ev1);
    case 1024: return p1_width_launch<T, 4, 8, 4, 1>(a, epi, ln, n, st, ev0, ev1);
    case 768: return p1_width_launch<T, 3, 8, 3, 1>(a, epi, ln, n, st, ev0, ev1);
    case 512: return p1_width_launch<T, 2, 8, 2, 1>(a, epi, ln, n, st, ev0, ev1);
    case 384: return p1_width_launch<T, 2, 4, 3, 1>(a, epi, ln, n, st, ev0, ev1);
    case 128: return p1_width_launch<T, 1, 4, 1, 1>(a, epi, ln, n, st, ev0, ev1);
    default: return -1;
  }
}

template int launch_proj1<float>(const GemmArgs&, int, bool, hipStream_t, hipEvent_t, hipEvent_t);
template int launch_proj1<half_t>(const GemmArgs&, int, bool, hipStream_t, hipEvent_t, hipEvent_t);

template int launch_proj_partial<float>(const GemmArgs&, int, hipStream_t, int*, hipEvent_t, hipEvent_t);
template int launch_proj_partial<half_t>(const GemmArgs&, int, hipStream_t, int*, hipEvent_t, hipEvent_t);

}  // namespace wh

#if WH_TUNING
WH_CT_READER(proj)
#endif
