// The per-date record and work layout of the grouped polish pipeline (polish_g.hip) and its
// wide-free-set solve (polish_gw.hip).
#pragma once
#include "common.h"
#include "../../include/porqua_hip.h"

namespace pq {

// per-date polish record (doubles), PQ_PG_RECORD in include/porqua_hip.h
constexpr int PGR = PQ_PG_RECORD;
enum : int {
  R_K = 0, R_MA = 1, R_NZB = 2, R_STATE = 3, R_ROUNDS = 4, R_SC = 5,
  // R_FORMED = 1: the K scratch holds P_FF of the free list of the last form (its positions
  // in PGWork::posF); R_REUSE = 1: this round's free list is a subset of it, so the round
  // gathers its P_FF from K instead of forming it again
  R_FORMED = 6, R_REUSE = 7,
  R_ACT = 64, R_LAM = 128, R_DA = 192, R_SOL = 256, R_AL = 288,
  // wide mode: R_W = 1 this round, R_NFX fixed variables at R_FIX (indices), R_FIXV (bound
  // values), R_FXL (their multipliers = box duals)
  R_W = 320, R_NFX = 321, R_FIX = 324, R_FIXV = 332, R_FXL = 340,
  // R_GFORM = g + 1: this round's P_FF comes from the group Gram (k_pg_form_grp) in the
  // pass scratch of the date's polish group g (0: the date forms alone)
  R_GFORM = 348,
  // R_KB: the free-set size setup found this round -- the LDS solve's buckets select on it
  // (the solve's inner primal loop lowers R_K while the other buckets may still be reading)
  R_KB = 349,
  // the solve buckets' date lists: record i holds at R_LIST + j the i-th date of bucket j (free
  // sets <= 48, 64, 80, 96, 128, and PG_BIGB: the large free sets of k_pg_big); date 0's record
  // holds the counts at R_CNT (as 64-bit integers, appended by k_pg_form's atomics, cleared by
  // k_pg_post<0>)
  R_LIST = 352, R_CNT = 360
};
constexpr int PG_NBUCKET = 6;
constexpr int PG_BIGB = 5;
__device__ __forceinline__ unsigned long long pg_count(const double* rec, int bk) {
  return reinterpret_cast<const unsigned long long*>(rec + R_CNT)[bk];
}
__device__ __forceinline__ int pg_listed(const double* rec, int bk, int i) {
  return (int)rec[(int64_t)i * PGR + R_LIST + bk];
}
// grid of a grid-stride kernel over at most B items: the workgroups that fit on the device at
// once (occupancy x CUs, queried once per kernel and device), at most B
int resident_grid(const void* kernel, int block, int B);
__device__ __forceinline__ int pg_bucket(int kb) {
  return kb <= 48 ? 0 : kb <= 64 ? 1 : kb <= 80 ? 2 : kb <= 96 ? 3 : 4;
}
constexpr int PG_KMAX = 128;   // largest free set of the LDS solve
constexpr int PG_KBIG = 256;   // largest free set of the grouped large-free-set solve (k_pg_big)
constexpr int PG_MGMAX = 32;   // general rows
// wide mode (polish_gw.hip): the free set exceeds the LDS solve, so the round solves the full
// n-space reduced KKT by the group capacitance with the active general rows and the fixed
// variables as bordered rows (at most PG_WMB of them)
constexpr int PG_WMB = 8;
constexpr int PG_WG_MAX = 24;   // general rows of the wide mode
static_assert(R_FXL + PG_WMB <= R_GFORM && R_KB < R_LIST && R_LIST + 6 <= R_CNT && R_CNT + 6 <= PQ_PG_RECORD,
              "PQ_PG_RECORD too small");

struct PGWork {   // per-date work layout: xs | xb | g | Px | Fl | rF | solx | pxb | U | fl
  double *xs, *xb, *g, *Px, *rF, *solx, *pxb, *U;
  int *Fl, *fl, *posF;   // posF (n ints, the upper half of Fl's slot): position of a variable
                         // in the free list of the last form, -1 when not in it
  __device__ __forceinline__ PGWork(const pq_state& st, int b, int ld) {
    double* W = st.work + (int64_t)b * st.work_stride;
    xs = W;
    xb = W + ld;
    g = W + 2 * (int64_t)ld;
    Px = W + 3 * (int64_t)ld;
    Fl = reinterpret_cast<int*>(W + 4 * (int64_t)ld);
    posF = Fl + ld;
    rF = W + 5 * (int64_t)ld;
    solx = W + 6 * (int64_t)ld;
    pxb = W + 7 * (int64_t)ld;
    U = W + 8 * (int64_t)ld;
    fl = reinterpret_cast<int*>(U + (int64_t)st.mg_pad * ld);
  }
};

__device__ __forceinline__ int pk(int r, int c) { return ((r * (r + 1)) >> 1) + c; }

}  // namespace pq

// wide rounds (polish_gw.hip), launched by pq_polish_grouped_round
// the register-tile solve (polish_rt.hip) of the free-set buckets <= 48 .. <= 16 nbmax (nbmax
// in 3..6), one launch
int pq_pg_solve_rt_launch(int nbmax, int B, hipStream_t str, const pq_problem* pb, pq_state* st, double* rec,
                          const pq_settings* s, int ldk);
int pq_pg_wide_launch(const pq_lowrank* lr, const pq_problem* pb, pq_state* st, double* rec, const pq_settings* s,
                      const pq_pg_wide* wd, hipStream_t stream);
