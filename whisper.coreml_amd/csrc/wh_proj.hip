// Launcher for k_proj (wh_proj.h): the split-K projections of the decoder step.
//
// Output format is the k_gemv_x EPI_PARTIAL one (fp32 slabs out_f32[z][M][N]), so the
// consumers (k_resid_ln, k_reduce_store, k_self_attn_qkv) are unchanged.  The tile
// configuration is picked per shape from a short list: rows in one row group when
// M <= 112 (MT = ceil(M/16)), then the configuration with the most workgroups that
// still fits one workgroup per CU (256) — measured on MI355X at 100 rows
// (tools/proj_bench.hip, profiles/r01/proj_bench.txt): qkv 4.0, out 6.0, fc1 / fc2 11.2
// -> 8.3 us per launch against k_gemv_x.
#include <cstdlib>

#include "wh_proj.h"

namespace wh {

namespace {

struct Cfg { int nsub, kw, nstep; };
constexpr Cfg CFGS[] = {{4, 1, 5}, {4, 1, 10}, {5, 1, 10}, {4, 1, 4}, {4, 1, 6}};
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
int launch_proj_partial(const GemmArgs& a, int max_z, hipStream_t st, int* z_out) {
  static Table<T> tab;
  static const bool off = [] {
    const char* e = getenv("WHISPER_HIP_PROJ");
    return e && e[0] == '0';
  }();
  if (off || a.M < 1 || a.M > 112 || a.K % 32 || a.N % 16 || a.x_group_rows < a.M) return -1;
  const int mt = (a.M + 15) / 16, S = a.K / 32;
  int best = -1, best_wgs = 0, best_z = 0;
  for (int c = 0; c < NCFG; ++c) {
    const Cfg& k = CFGS[c];
    if (S % (k.kw * k.nstep)) continue;
    const int z = S / (k.kw * k.nstep);
    if (z > max_z || z > 16 || tab.e[mt - 1][c].lds > LDS_MAX) continue;
    const int wgs = (a.N + 16 * k.nsub - 1) / (16 * k.nsub) * z;
    if (wgs > 256) continue;
    if (wgs > best_wgs || (wgs == best_wgs && k.nstep > CFGS[best].nstep)) best = c, best_wgs = wgs, best_z = z;
  }
  if (best < 0) return -1;
  const Ent& e = tab.e[mt - 1][best];
  if (!tab.attr[mt - 1][best]) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(e.f), hipFuncAttributeMaxDynamicSharedMemorySize, e.lds) !=
        hipSuccess)
      return -2;
    tab.attr[mt - 1][best] = true;
  }
  GemmArgs b = a;
  b.ksplit = best_z;
  hipLaunchKernelGGL(e.f, dim3(best_wgs), dim3(64 * CFGS[best].nsub * CFGS[best].kw), e.lds, st, b);
  *z_out = best_z;
  return 0;
}

template int launch_proj_partial<float>(const GemmArgs&, int, hipStream_t, int*);
template int launch_proj_partial<half_t>(const GemmArgs&, int, hipStream_t, int*);

}  // namespace wh
