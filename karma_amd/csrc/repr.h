// repr.h — Python repr() of a double, on the device and the host.
//
// ReadGraph.edge_list (karma/read_graph.py:350-357) writes every weight with
// an f-string, i.e. CPython's repr(float): the SHORTEST decimal digit string
// that reads back as the same double (closest to it among the shortest, ties
// to an even last digit), laid out by float_repr_style 'short' rules:
//   decpt = position of the decimal point relative to the digits;
//   -4 < decpt <= 16 : fixed notation, "0.000ddd", "dd.ddd", "ddd00.0";
//   otherwise        : "d.ddde-05" / "de+16" (sign, at least two exponent digits).
// The shortest digits come from the Ryu algorithm (Ulf Adams, "Ryu: fast
// float-to-string conversion", PLDI 2018), restated here on 128-bit products
// of the mantissa with the power-of-5 tables of repr_tables.h.  Parity with
// CPython is tested on the host build of this header (tests/test_repr_cpu.py)
// and through the edge-list kernel on the GPU.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "repr_tables.h"

namespace karma_repr {

constexpr int kPow5Bits = 125;
constexpr int kPow5InvBits = 125;
constexpr int kMaxRepr = 32;  // longest repr of a double ("-2.2250738585072014e-308" is 24)

__host__ __device__ inline uint32_t pow5bits(int32_t e) { return (uint32_t)(((uint32_t)e * 1217359u) >> 19) + 1u; }
__host__ __device__ inline uint32_t log10_pow2(int32_t e) { return ((uint32_t)e * 78913u) >> 18; }
__host__ __device__ inline uint32_t log10_pow5(int32_t e) { return ((uint32_t)e * 732923u) >> 20; }

__host__ __device__ inline uint32_t pow5_factor(uint64_t v) {
    uint32_t n = 0;
    for (;;) {
        const uint64_t q = v / 5, r = v - 5 * q;
        if (r != 0) break;
        v = q;
        ++n;
    }
    return n;
}
__host__ __device__ inline bool multiple_of_pow5(uint64_t v, uint32_t p) { return pow5_factor(v) >= p; }
__host__ __device__ inline bool multiple_of_pow2(uint64_t v, uint32_t p) { return (v & ((1ull << p) - 1)) == 0; }

// (m * mul) >> j for a 128-bit multiplier {lo, hi}, j >= 64, m < 2^55
__host__ __device__ inline uint64_t mul_shift64(uint64_t m, const uint64_t* mul, int32_t j) {
    const unsigned __int128 b0 = (unsigned __int128)m * mul[0];
    const unsigned __int128 b2 = (unsigned __int128)m * mul[1];
    return (uint64_t)(((b0 >> 64) + b2) >> (j - 64));
}

struct Decimal {
    uint64_t digits;  // shortest digit string as an integer
    int32_t exp10;    // value = digits * 10^exp10
};

// Shortest round-trip decimal of a positive finite double (mantissa bits,
// biased exponent), Ryu's d2d.
__host__ __device__ inline Decimal shortest(uint64_t ieee_m, uint32_t ieee_e) {
    int32_t e2;
    uint64_t m2;
    if (ieee_e == 0) {
        e2 = 1 - 1023 - 52 - 2;
        m2 = ieee_m;
    } else {
        e2 = (int32_t)ieee_e - 1023 - 52 - 2;
        m2 = (1ull << 52) | ieee_m;
    }
    const bool accept_bounds = (m2 & 1) == 0;  // round-half-even reading keeps even mantissas' bounds
    const uint64_t mv = 4 * m2;
    const uint32_t mm_shift = ieee_m != 0 || ieee_e <= 1;  // the gap below is half as wide at 2^k
    uint64_t vr, vp, vm;
    int32_t e10;
    bool vm_tz = false, vr_tz = false;
    if (e2 >= 0) {
        const uint32_t q = log10_pow2(e2) - (e2 > 3);
        e10 = (int32_t)q;
        const int32_t k = kPow5InvBits + (int32_t)pow5bits((int32_t)q) - 1;
        const int32_t i = -e2 + (int32_t)q + k;
        vr = mul_shift64(4 * m2, kPow5Inv[q], i);
        vp = mul_shift64(4 * m2 + 2, kPow5Inv[q], i);
        vm = mul_shift64(4 * m2 - 1 - mm_shift, kPow5Inv[q], i);
        if (q <= 21) {
            if (mv % 5 == 0) vr_tz = multiple_of_pow5(mv, q);
            else if (accept_bounds) vm_tz = multiple_of_pow5(mv - 1 - mm_shift, q);
            else vp -= multiple_of_pow5(mv + 2, q);
        }
    } else {
        const uint32_t q = log10_pow5(-e2) - (-e2 > 1);
        e10 = (int32_t)q + e2;
        const int32_t i = -e2 - (int32_t)q;
        const int32_t k = (int32_t)pow5bits(i) - kPow5Bits;
        const int32_t j = (int32_t)q - k;
        vr = mul_shift64(4 * m2, kPow5[i], j);
        vp = mul_shift64(4 * m2 + 2, kPow5[i], j);
        vm = mul_shift64(4 * m2 - 1 - mm_shift, kPow5[i], j);
        if (q <= 1) {
            vr_tz = true;
            if (accept_bounds) vm_tz = mm_shift == 1;
            else --vp;
        } else if (q < 63) {
            vr_tz = multiple_of_pow2(mv, q);
        }
    }
    int32_t removed = 0;
    uint32_t last = 0;
    uint64_t out;
    if (vm_tz || vr_tz) {
        // general case: track whether the removed digits were all zero
        for (;;) {
            const uint64_t vp10 = vp / 10, vm10 = vm / 10;
            if (vp10 <= vm10) break;
            const uint32_t vm_mod = (uint32_t)(vm - 10 * vm10);
            const uint64_t vr10 = vr / 10;
            const uint32_t vr_mod = (uint32_t)(vr - 10 * vr10);
            vm_tz &= vm_mod == 0;
            vr_tz &= last == 0;
            last = vr_mod;
            vr = vr10;
            vp = vp10;
            vm = vm10;
            ++removed;
        }
        if (vm_tz) {
            for (;;) {
                const uint64_t vm10 = vm / 10;
                const uint32_t vm_mod = (uint32_t)(vm - 10 * vm10);
                if (vm_mod != 0) break;
                const uint64_t vp10 = vp / 10, vr10 = vr / 10;
                const uint32_t vr_mod = (uint32_t)(vr - 10 * vr10);
                vr_tz &= last == 0;
                last = vr_mod;
                vr = vr10;
                vp = vp10;
                vm = vm10;
                ++removed;
            }
        }
        if (vr_tz && last == 5 && vr % 2 == 0) last = 4;  // exactly ...50..0: round half to even
        out = vr + ((vr == vm && (!accept_bounds || !vm_tz)) || last >= 5);
    } else {
        bool round_up = false;
        const uint64_t vp100 = vp / 100, vm100 = vm / 100;
        if (vp100 > vm100) {
            const uint64_t vr100 = vr / 100;
            const uint32_t vr_mod = (uint32_t)(vr - 100 * vr100);
            round_up = vr_mod >= 50;
            vr = vr100;
            vp = vp100;
            vm = vm100;
            removed += 2;
        }
        for (;;) {
            const uint64_t vp10 = vp / 10, vm10 = vm / 10;
            if (vp10 <= vm10) break;
            const uint64_t vr10 = vr / 10;
            const uint32_t vr_mod = (uint32_t)(vr - 10 * vr10);
            round_up = vr_mod >= 5;
            vr = vr10;
            vp = vp10;
            vm = vm10;
            ++removed;
        }
        out = vr + (vr == vm || round_up);
    }
    return Decimal{out, e10 + removed};
}

// repr(x) as (sign, digit string, decimal point) and the layout rules, with no
// local arrays: device code keeps everything in registers (a char buffer would
// live in scratch memory, one slow round trip per byte).
struct Parts {
    int kind;         // 0 nan, 1 inf, 2 finite
    bool neg;
    uint64_t digits;  // shortest digits as an integer ("0" for zero)
    int nd;           // their number
    int32_t decpt;    // decimal point position relative to the digits
};

__host__ __device__ inline Parts parts(double x) {
    Parts p;
    const uint64_t bits = __builtin_bit_cast(uint64_t, x);
    p.neg = (bits >> 63) != 0;
    const uint64_t ieee_m = bits & ((1ull << 52) - 1);
    const uint32_t ieee_e = (uint32_t)((bits >> 52) & 0x7FF);
    p.digits = 0;
    p.nd = 1;
    p.decpt = 1;
    if (ieee_e == 0x7FF) {
        p.kind = ieee_m ? 0 : 1;
        return p;
    }
    p.kind = 2;
    if (ieee_e == 0 && ieee_m == 0) return p;  // "0.0"
    const Decimal d = shortest(ieee_m, ieee_e);
    p.digits = d.digits;
    uint64_t t = 10;
    while (p.nd < 19 && d.digits >= t) {  // at most 17 digits
        ++p.nd;
        t *= 10;
    }
    p.decpt = d.exp10 + p.nd;
    return p;
}

__host__ __device__ inline int parts_len(const Parts& p) {
    if (p.kind == 0) return 3;                   // nan (repr drops the sign)
    if (p.kind == 1) return 3 + (p.neg ? 1 : 0);  // inf, -inf
    int n = p.neg ? 1 : 0;
    if (p.decpt <= -4 || p.decpt > 16) {  // d.ddde-05
        int ex = p.decpt - 1;
        ex = ex < 0 ? -ex : ex;
        return n + 1 + (p.nd > 1 ? p.nd : 0) + 2 + (ex >= 100 ? 3 : 2);
    }
    if (p.decpt <= 0) return n + 2 - p.decpt + p.nd;  // 0.000ddd
    if (p.decpt < p.nd) return n + p.nd + 1;          // dd.ddd
    return n + p.decpt + 2;                           // ddd00.0
}

// writes parts_len(p) bytes at dst (any address space)
template <typename Out>
__host__ __device__ inline void parts_write(const Parts& p, Out* dst) {
    if (p.kind == 0) {
        dst[0] = 'n', dst[1] = 'a', dst[2] = 'n';
        return;
    }
    int o = 0;
    if (p.neg) dst[o++] = '-';
    if (p.kind == 1) {
        dst[o] = 'i', dst[o + 1] = 'n', dst[o + 2] = 'f';
        return;
    }
    const int nd = p.nd, dp = p.decpt;
    const bool expo = dp <= -4 || dp > 16;
    // digit t (0 = most significant) goes to o + pos(t); written last to first
    uint64_t v = p.digits;
    for (int t = nd - 1; t >= 0; --t) {
        const uint64_t q = v / 10;
        const char ch = (char)('0' + (uint32_t)(v - 10 * q));
        v = q;
        int pos;
        if (expo) pos = t == 0 ? 0 : t + 1;
        else if (dp <= 0) pos = 2 - dp + t;
        else pos = t < dp ? t : t + 1;
        dst[o + pos] = ch;
    }
    if (expo) {
        int n = o + 1;
        if (nd > 1) {
            dst[o + 1] = '.';
            n = o + nd + 1;
        }
        int ex = dp - 1;
        dst[n++] = 'e';
        dst[n++] = ex < 0 ? '-' : '+';
        if (ex < 0) ex = -ex;
        if (ex >= 100) dst[n++] = (char)('0' + ex / 100);
        dst[n++] = (char)('0' + (ex / 10) % 10);
        dst[n] = (char)('0' + ex % 10);
    } else if (dp <= 0) {
        dst[o] = '0';
        dst[o + 1] = '.';
        for (int t = 0; t < -dp; ++t) dst[o + 2 + t] = '0';
    } else if (dp < nd) {
        dst[o + dp] = '.';
    } else {
        for (int t = nd; t < dp; ++t) dst[o + t] = '0';
        dst[o + dp] = '.';
        dst[o + dp + 1] = '0';
    }
}

// Writes repr(x) (no terminator) to dst, returns its length (<= kMaxRepr).
// dst == nullptr: length only.
__host__ __device__ inline int repr_f64(double x, char* dst) {
    const Parts p = parts(x);
    if (dst) parts_write(p, dst);
    return parts_len(p);
}

}  // namespace karma_repr
