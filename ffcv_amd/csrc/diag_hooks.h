// diag_hooks.h -- hooks of the timing-only diagnostic builds (tools/
// build_variant.sh, tools/k1_phase_valu.sh, tools/jpeg_phases.py).  In the
// product build (ffcv_amd/_build.py) every hook compiles to nothing.
//
//   -DK1_STOP=n      K1 returns at phase-end hook n (its output is then
//                    wrong: only the time or counters up to that point count)
//   -DFFCV_K1_DIAG   K1's decode loops count their iterations (two
//                    instructions per step) for tools/jpeg_phases.py
//   -DRRC_STOP=n     the raw RRC kernel returns at hook n (wrong output)
//   -DK2_STOP=n      the per-band K2's linear fast path returns at hook n
#pragma once

#ifdef K1_STOP
// `cond` is an opaque always-true test, so the compiler keeps the code after
// the stop point and the stop build's instruction layout stays comparable
#define K1_STOP_AT(n, cond, ...) \
  if (K1_STOP == (n) && (cond)) return __VA_ARGS__
#else
#define K1_STOP_AT(n, cond, ...) \
  do {                            \
  } while (0)
#endif

#ifdef FFCV_K1_DIAG
#define K1_DIAG(x) x
#else
#define K1_DIAG(x)
#endif

#ifdef RRC_STOP
#define RRC_STOP_AT(n, cond, ...) \
  if (RRC_STOP == (n) && (cond)) return __VA_ARGS__
#else
#define RRC_STOP_AT(n, cond, ...) \
  do {                             \
  } while (0)
#endif

#ifdef K2_STOP
#define K2_STOP_AT(n, cond, ...) \
  if (K2_STOP == (n) && (cond)) return __VA_ARGS__
#else
#define K2_STOP_AT(n, cond, ...) \
  do {                            \
  } while (0)
#endif
