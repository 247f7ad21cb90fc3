// bg_map.hip — K5: bedmap <ops> ref map with the default overlap rule (--bp-ovr N).
//
// Reference: WindowSweep::sweep overload 2 (interfaces/src/algorithm/sweep/
// WindowSweepImpl.cpp:168-256) keeps a deque window of map rows; BedBaseVisitor::
// fixWindow (algorithm/visitors/bed/BedBaseVisitor.hpp:184-215) re-tests the window
// against each reference row with Overlapping(N) (data/bed/BedDistances.hpp:95-115),
// and Count / Average (numerical/CountVisitor.hpp, AverageVisitor.hpp) accumulate.
// For every reference row r that yields the multiset
//   S(r) = { m : same chrom, min(r.e, m.e) - max(r.s, m.s) >= N }
// (verified by randomized differential tests against the reference).
// GPU form: map rows are start-sorted, so with L = max map length (computed by the
// loader) every m in S(r)
// has m.s in [r.s - L + 1, r.e): two binary searches bound the candidates, one
// thread per reference row accumulates count and the exact integer score sum.
// Exactness: the reference keeps ONE running double across the file
// (AverageVisitor.hpp:46-54); it equals our exact per-row sum whenever scores are
// integers and partial sums stay below 2^53. Other inputs are refused
// (BG_E_UNSUPPORTED) rather than approximated; so are zero-length rows, on which the
// reference's stream consumption differs from S(r).
#include <climits>

#include "bg_internal.h"

__global__ void __launch_bounds__(BG_NT) k_map_count_sum(
    const int64_t* __restrict__ RS, const int64_t* __restrict__ RE, uint64_t nr,
    const int64_t* __restrict__ MS, const int64_t* __restrict__ ME, const double* __restrict__ SC,
    uint64_t nm, int64_t L, int64_t ovr, int32_t* __restrict__ cnt, int64_t* __restrict__ isum,
    bg_dstatus* st) {
  const uint64_t r = (uint64_t)blockIdx.x * BG_NT + threadIdx.x;
  if (r >= nr) return;
  const int64_t s = RS[r], e = RE[r];
  const uint64_t lo = lower_bound_i64(MS, nm, s - L + 1);
  const uint64_t hi = lower_bound_i64(MS, nm, e);
  int32_t c = 0;
  int64_t sum = 0;
  for (uint64_t m = lo; m < hi; ++m) {
    const int64_t ov = min(e, ME[m]) - max(s, MS[m]);
    if (ov >= ovr) {
      ++c;
      if (SC) sum += (int64_t)SC[m];
    }
  }
  cnt[r] = c;
  if (isum) {
    isum[r] = sum;
    if (sum >= (1LL << 53) || sum <= -(1LL << 53)) atomicOr(&st->flags, 4ULL);
  }
}

extern "C" int bg_map(bg_ctx* c, bg_set* set, int ref, int map, const bg_map_opts* opts,
                      bg_result** out) {
  if (!c || !set || !opts || !out || ref < 0 || map < 0 || ref >= (int)set->t.size() ||
      map >= (int)set->t.size() || opts->n_ops <= 0 || opts->n_ops > 16)
    return BG_E_ARG;
  {
    const int f[2] = {ref, map};
    int rc0 = bg_need_rows(c, set, f, 2, "bedmap");
    if (rc0) return rc0;
  }
  bool need_score = false;
  for (int k = 0; k < opts->n_ops; ++k) {
    if (opts->ops[k] == BG_MAP_MEAN) need_score = true;
    else if (opts->ops[k] != BG_MAP_COUNT) return bg_fail(c, BG_E_UNSUPPORTED, "bedmap operation not on the GPU path");
  }
  if (opts->scientific) return bg_fail(c, BG_E_UNSUPPORTED, "--sci is not on the GPU path yet");
  if (opts->precision < 0 || opts->precision > 17) return bg_fail(c, BG_E_UNSUPPORTED, "--prec above 17 is not on the GPU path");
  if (opts->overlap_bp < 1) return BG_E_ARG;
  bg_table* R = set->t[ref];
  bg_table* M = set->t[map];
  if (need_score && (M->kind != BG_BED5 || !M->score)) return bg_fail(c, BG_E_ARG, "--mean needs the map file loaded as BG_BED5");
  if (R->has_zero_len || M->has_zero_len)
    return bg_fail(c, BG_E_UNSUPPORTED, "zero-length elements (end == start) are not on the GPU path of bedmap");
  if (need_score && !M->score_int)
    return bg_fail(c, BG_E_UNSUPPORTED, "non-integer map scores are not on the GPU path of bedmap --mean yet");
  BG_HIP(c, hipMemsetAsync(c->dstat, 0, sizeof(bg_dstatus), c->stream));
  int32_t* cnt = (int32_t*)bg_alloc(c, 4 * (R->n ? R->n : 1));
  int64_t* isum = need_score ? (int64_t*)bg_alloc(c, 8 * (R->n ? R->n : 1)) : nullptr;
  if (!cnt || (need_score && !isum)) return BG_E_NOMEM;
  const int64_t L = M->maxlen > 0 ? M->maxlen : 1;  // longest map row (from the loader)
  if (R->n)
    BG_LAUNCH(c, "k_map_count_sum", k_map_count_sum, dim3(bg_blocks(R->n, BG_NT)), dim3(BG_NT),
                       R->ks, R->ke, R->n, M->ks, M->ke, need_score ? M->score : nullptr, M->n, L,
                       (int64_t)opts->overlap_bp, cnt, isum, c->dstat);
  BG_HIP(c, hipGetLastError());
  BG_HIP(c, hipMemcpyAsync(c->hstat, c->dstat, sizeof(bg_dstatus), hipMemcpyDeviceToHost, c->stream));
  BG_HIP(c, hipStreamSynchronize(c->stream));
  if (c->hstat->flags & 4ULL)
    return bg_fail(c, BG_E_UNSUPPORTED, "a window score sum reaches 2^53 (inexact in the reference too)");
  bg_result* res = new bg_result();
  res->ctx = c;
  res->set = set;
  res->kind = RES_MAP;
  res->n = R->n;
  res->cnt = cnt;
  res->isum = isum;
  res->mopts = *opts;
  res->tab = ref;
  *out = res;
  bg_mark(c, "map");
  return 0;
}
