// ABI introspection for the ctypes binding (sizeof / offsetof of the arg structs).
#include <hip/hip_runtime.h>
#include "args.h"

#define FM_OFF(S, f) if (!__builtin_strcmp(field, #f)) return (long long)offsetof(S, f)

extern "C" long long fm_abi_sizeof(const char* name) {
  if (!__builtin_strcmp(name, "DetectArgs")) return sizeof(DetectArgs);
  if (!__builtin_strcmp(name, "SmoothArgs")) return sizeof(SmoothArgs);
  if (!__builtin_strcmp(name, "RankArgs")) return sizeof(RankArgs);
  if (!__builtin_strcmp(name, "WindowArgs")) return sizeof(WindowArgs);
  if (!__builtin_strcmp(name, "BivArgs")) return sizeof(BivArgs);
  return -1;
}

extern "C" long long fm_abi_offsetof(const char* name, const char* field) {
  if (!__builtin_strcmp(name, "SmoothArgs")) { FM_OFF(SmoothArgs, det); FM_OFF(SmoothArgs, season_out); FM_OFF(SmoothArgs, grid); FM_OFF(SmoothArgs, head_dev); FM_OFF(SmoothArgs, season_hb); FM_OFF(SmoothArgs, nvalid_out); }
  if (!__builtin_strcmp(name, "DetectArgs")) { FM_OFF(DetectArgs, pw_scale); FM_OFF(DetectArgs, app_stats); FM_OFF(DetectArgs, ld_cur);
    FM_OFF(DetectArgs, threshold_low); FM_OFF(DetectArgs, hv_grid); FM_OFF(DetectArgs, hv_m); FM_OFF(DetectArgs, forecast);
    FM_OFF(DetectArgs, anom_count); FM_OFF(DetectArgs, anom_cap); FM_OFF(DetectArgs, thr_lut); FM_OFF(DetectArgs, lut_n);
    FM_OFF(DetectArgs, row_out); FM_OFF(DetectArgs, tick_min); FM_OFF(DetectArgs, shift_one_step); }
  if (!__builtin_strcmp(name, "RankArgs")) { FM_OFF(RankArgs, pvals); FM_OFF(RankArgs, alpha); FM_OFF(RankArgs, p_friedman); FM_OFF(RankArgs, pods_b); FM_OFF(RankArgs, z_crit); }
  if (!__builtin_strcmp(name, "WindowArgs")) { FM_OFF(WindowArgs, det); }
  if (!__builtin_strcmp(name, "BivArgs")) { FM_OFF(BivArgs, eps); FM_OFF(BivArgs, app_stats); }
  return -1;
}
