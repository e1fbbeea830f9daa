/*
 * dragg_results.h -- C ABI of the host-side results formatter (libdragg_results.so).
 *
 *   reference                                   this ABI
 *   -----------------------------------------   ------------------------------------------
 *   write_outputs: json.dump(collected, f,      dragg_fmt_series() renders every list of floats
 *     indent=4)            aggregator.py:839      of the document; dragg_amd/results.py lays out
 *   all_homes-N-config.json json.dump(...,          the structure around them (json.dump's indent=4
 *     indent=4)            aggregator.py:846      layout, byte for byte)
 *
 * Numbers are rendered as Python's repr(float) (json.dump's float spelling): the shortest digits that
 * round-trip, fixed notation for decimal-point positions -4 < decpt <= 16, else d.ddde+XX (at least two
 * exponent digits), "NaN", "Infinity", "-Infinity".  Host memory only; no GPU.
 */
#ifndef DRAGG_RESULTS_H
#define DRAGG_RESULTS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DRAGG_RESULTS_ABI_VERSION 1
/* bytes one number may take (sign, 17 digits, point, exponent) */
#define DRAGG_FMT_MAX 32

int dragg_results_abi_version(void);

/* One double as repr(float) into out (>= DRAGG_FMT_MAX bytes, not terminated); returns its length. */
int64_t dragg_fmt_double(double v, char* out);

/* n_series lists of doubles: list s = x[begin[s] .. end[s]), rendered with `sep` (sep_len bytes) between
   its numbers, written at out + out_starts[s] (the caller reserves (count * (DRAGG_FMT_MAX + sep_len))
   bytes per list), its length in out_len[s].  Lists are formatted in parallel (OpenMP).  Returns 0, or
   -1 on a bad argument. */
int64_t dragg_fmt_series(const double* x, const int64_t* begin, const int64_t* end, int64_t n_series, const char* sep,
                         int64_t sep_len, char* out, const int64_t* out_starts, int64_t* out_len);

#ifdef __cplusplus
}
#endif
#endif /* DRAGG_RESULTS_H */
