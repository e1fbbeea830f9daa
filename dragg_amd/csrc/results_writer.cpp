// results_writer.cpp -- host-side number formatting of the run's output files.
//
// The reference writes results.json and all_homes-N-config.json with json.dump(..., indent=4)
// (aggregator.py:839-854): at 10k homes x 96 steps that is ~25 M floats, each rendered by Python's
// pure-Python indenting encoder (float.__repr__ per number and a file write per token) -- over a
// minute per results.json, far longer than the 96 device steps it records.  dragg_amd/results.py keeps
// the document's structure in Python and hands every list of floats to this library, which renders
// the numbers exactly as float.__repr__ does (the shortest digits that round-trip, laid out by
// CPython's repr rule: fixed notation for decimal exponents -4 < decpt <= 16, else d.ddde+XX) with
// json.dump's spellings NaN / Infinity / -Infinity, joined by the list separator -- the same bytes,
// OpenMP-parallel over the lists.  Built with g++ (dragg_amd/build.py); no GPU code.
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/dragg_results.h"

// sha-256 of this file and its header, stamped by dragg_amd/build.py (a stale build is rebuilt)
#ifndef DRAGG_RESULTS_SOURCE_HASH
#define DRAGG_RESULTS_SOURCE_HASH "unstamped"
#endif
extern "C" const char dragg_results_stamp[] = "dragg-results-sha256:" DRAGG_RESULTS_SOURCE_HASH;

namespace {

// one double as Python's repr(float) (json.dump's float spelling for non-finite values)
int fmt_double(double v, char* out) {
    if (std::isnan(v)) { std::memcpy(out, "NaN", 3); return 3; }
    if (std::isinf(v)) {
        if (v > 0) { std::memcpy(out, "Infinity", 8); return 8; }
        std::memcpy(out, "-Infinity", 9);
        return 9;
    }
    char buf[40];
    // shortest round-trip digits in scientific form: [-]d[.ddd]e(+|-)XX
    const auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);
    const char* p = buf;
    const char* end = r.ptr;
    char* o = out;
    if (*p == '-') { *o++ = '-'; ++p; }
    char dig[24];
    int nd = 0;
    for (; p < end && *p != 'e'; ++p)
        if (*p != '.') dig[nd++] = *p;
    int e = 0;
    if (p < end) {                                   // the exponent
        ++p;
        bool neg = false;
        if (*p == '+' || *p == '-') { neg = *p == '-'; ++p; }
        for (; p < end; ++p) e = e * 10 + (*p - '0');
        if (neg) e = -e;
    }
    while (nd > 1 && dig[nd - 1] == '0') --nd;      // (shortest form has none; kept for safety)
    const int decpt = e + 1;                         // digits d1 d2 ... with the point after decpt of them
    if (decpt <= -4 || decpt > 16) {                 // CPython's repr: exponent notation
        *o++ = dig[0];
        if (nd > 1) {
            *o++ = '.';
            std::memcpy(o, dig + 1, nd - 1);
            o += nd - 1;
        }
        *o++ = 'e';
        *o++ = e < 0 ? '-' : '+';
        const int a = e < 0 ? -e : e;
        if (a >= 100) { *o++ = char('0' + a / 100); *o++ = char('0' + a / 10 % 10); *o++ = char('0' + a % 10); }
        else { *o++ = char('0' + a / 10); *o++ = char('0' + a % 10); }
    } else if (decpt <= 0) {                         // 0.000ddd
        *o++ = '0';
        *o++ = '.';
        for (int i = 0; i < -decpt; ++i) *o++ = '0';
        std::memcpy(o, dig, nd);
        o += nd;
    } else if (decpt >= nd) {                        // ddd000.0
        std::memcpy(o, dig, nd);
        o += nd;
        for (int i = nd; i < decpt; ++i) *o++ = '0';
        *o++ = '.';
        *o++ = '0';
    } else {                                         // ddd.ddd
        std::memcpy(o, dig, decpt);
        o += decpt;
        *o++ = '.';
        std::memcpy(o, dig + decpt, nd - decpt);
        o += nd - decpt;
    }
    return int(o - out);
}

}  // namespace

extern "C" {

int dragg_results_abi_version(void) { return DRAGG_RESULTS_ABI_VERSION; }

int64_t dragg_fmt_double(double v, char* out) { return fmt_double(v, out); }

int64_t dragg_fmt_series(const double* x, const int64_t* begin, const int64_t* end, int64_t n_series, const char* sep,
                         int64_t sep_len, char* out, const int64_t* out_starts, int64_t* out_len) {
    if (n_series < 0 || (n_series > 0 && (!x || !begin || !end || !out || !out_starts || !out_len)) || sep_len < 0 ||
        (sep_len > 0 && !sep))
        return -1;
    int64_t bad = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : bad)
    for (int64_t s = 0; s < n_series; ++s) {
        const int64_t a = begin[s], b = end[s];
        if (b < a) { out_len[s] = 0; ++bad; continue; }
        char* o = out + out_starts[s];
        for (int64_t i = a; i < b; ++i) {
            if (i > a) { std::memcpy(o, sep, (size_t)sep_len); o += sep_len; }
            o += fmt_double(x[i], o);
        }
        out_len[s] = o - (out + out_starts[s]);
    }
    return bad ? -1 : 0;
}

}  // extern "C"
