// yc_num.h — exact conversions between decimal text and IEEE binary64, for the JSON numbers of
// ContentJSON / ContentEmbed / ContentFormat values (Y@72137 readContentJSON → JSON.parse, Y@71991
// write → JSON.stringify). Yjs keeps the parsed value, so a number comes back out as
// Number::toString of the double JSON.parse made of it:
//   dec_to_f64  JSON.parse's number: the double nearest the decimal value, ties to an even
//               significand (ECMA-262 RoundMVResult). Exact for any digit count: the first 800
//               significant digits decide (a binary64 halfway point has at most 767) and the rest
//               only say "above" (sticky).
//   f64_shortest Number::toString's digits: the fewest decimal digits that read back as the same
//               double, the candidate nearest the value when several have that many, an even last
//               digit on an exact tie (Steele & White's free-format algorithm with the interval
//               bounds closed for an even significand — the bignum fallback V8 uses).
// Both run on fixed-size big integers (no allocation), the same code on the host (the update
// scanner, tests) and on the device (k_json_canon). Rare path: only values whose text is not
// already in toString's form get here.
#pragma once
#include <cstdint>

namespace yc {

template <int L>
struct BigN {
  uint32_t n;  // limbs in use (no leading zero limb)
  uint32_t d[L];
};
template <int L>
YC_HDI void big_set(BigN<L>& a, uint64_t v) {
  a.n = 0;
  while (v) { a.d[a.n++] = (uint32_t)v; v >>= 32; }
}
template <int L>
YC_HD inline bool big_mul_small(BigN<L>& a, uint32_t m, uint32_t add = 0) {
  uint64_t c = add;
  for (uint32_t i = 0; i < a.n; ++i) {
    const uint64_t t = (uint64_t)a.d[i] * m + c;
    a.d[i] = (uint32_t)t;
    c = t >> 32;
  }
  if (c) {
    if (a.n == (uint32_t)L) return false;
    a.d[a.n++] = (uint32_t)c;
  }
  return true;
}
template <int L>
YC_HD inline bool big_shl(BigN<L>& a, uint32_t k) {
  if (a.n == 0 || k == 0) return true;
  const uint32_t w = k >> 5, s = k & 31u;
  const uint32_t top = s ? (a.d[a.n - 1] >> (32 - s)) : 0u;
  const uint32_t nn = a.n + w + (top ? 1u : 0u);
  if (nn > (uint32_t)L) return false;
  if (top) a.d[a.n + w] = top;
  for (uint32_t i = a.n; i-- > 0;) {
    const uint32_t lo = (s && i) ? (a.d[i - 1] >> (32 - s)) : 0u;
    a.d[i + w] = s ? ((a.d[i] << s) | lo) : a.d[i];
  }
  for (uint32_t i = 0; i < w; ++i) a.d[i] = 0;
  a.n = nn;
  return true;
}
template <int L>
YC_HD inline bool big_mul_pow5(BigN<L>& a, uint32_t k) {
  constexpr uint32_t P13 = 1220703125u;  // 5^13, the largest power of 5 in a limb
  for (; k >= 13; k -= 13)
    if (!big_mul_small(a, P13)) return false;
  uint32_t m = 1;
  for (; k; --k) m *= 5;
  return m == 1 || big_mul_small(a, m);
}
template <int L>
YC_HD inline int big_cmp(const BigN<L>& a, const BigN<L>& b) {
  if (a.n != b.n) return a.n < b.n ? -1 : 1;
  for (uint32_t i = a.n; i-- > 0;)
    if (a.d[i] != b.d[i]) return a.d[i] < b.d[i] ? -1 : 1;
  return 0;
}
template <int L>
YC_HD inline bool big_add(BigN<L>& a, const BigN<L>& b) {  // a += b
  const uint32_t n = a.n > b.n ? a.n : b.n;
  uint64_t c = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t t = (uint64_t)(i < a.n ? a.d[i] : 0u) + (i < b.n ? b.d[i] : 0u) + c;
    a.d[i] = (uint32_t)t;
    c = t >> 32;
  }
  a.n = n;
  if (c) {
    if (a.n == (uint32_t)L) return false;
    a.d[a.n++] = 1u;
  }
  return true;
}
template <int L>
YC_HD inline void big_sub(BigN<L>& a, const BigN<L>& b) {  // a -= b (a >= b)
  int64_t c = 0;
  for (uint32_t i = 0; i < a.n; ++i) {
    const int64_t t = (int64_t)a.d[i] - (i < b.n ? (int64_t)b.d[i] : 0) + c;
    a.d[i] = (uint32_t)t;
    c = t < 0 ? -1 : 0;
  }
  while (a.n && a.d[a.n - 1] == 0) --a.n;
}
// a + b compared with c
template <int L>
YC_HD inline int big_plus_cmp(const BigN<L>& a, const BigN<L>& b, const BigN<L>& c, BigN<L>& t) {
  t = a;
  if (!big_add(t, b)) return 1;
  return big_cmp(t, c);
}

YC_HDI uint64_t f64_bits(double x) { union { double d; uint64_t u; } c; c.d = x; return c.u; }
YC_HDI double f64_from(uint64_t u) { union { uint64_t u; double d; } c; c.u = u; return c.d; }
// a finite double >= 0 as m * 2^q (m < 2^53, q >= -1074)
YC_HDI void f64_split(uint64_t bits, uint64_t& m, int32_t& q) {
  const uint32_t be = (uint32_t)(bits >> 52) & 0x7FFu;
  m = bits & ((1ull << 52) - 1);
  if (be) { m |= 1ull << 52; q = (int32_t)be - 1075; } else { q = -1074; }
}

constexpr uint32_t DEC_MAX_DIGITS = 800;  // significant digits that decide the rounding (>= 767)
constexpr int DEC_LIMBS = 100;            // 3 200 bits: 10^800 times the scale factors below
using BigD = BigN<DEC_LIMBS>;

// D * 10^E (+ a nonzero tail when sticky) compared with (2m + 1) * 2^(q - 1), the midpoint between
// m * 2^q and (m + 1) * 2^q: -1 below, 0 at, 1 above. false on overflow of the limbs (never for
// the ranges dec_to_f64 passes).
YC_HD inline bool dec_cmp_mid(const BigD& D, int32_t E, bool sticky, uint64_t m, int32_t q, BigD& l, BigD& r, int& res) {
  // D * 5^E * 2^E  vs  (2m + 1) * 2^(q - 1)
  l = D;
  big_set(r, 2 * m + 1);
  int32_t p2 = E - (q - 1);  // power of two on the left, relative to the right
  if (E >= 0) {
    if (!big_mul_pow5(l, (uint32_t)E)) return false;
  } else {
    if (!big_mul_pow5(r, (uint32_t)-E)) return false;
  }
  if (p2 >= 0) { if (!big_shl(l, (uint32_t)p2)) return false; }
  else if (!big_shl(r, (uint32_t)-p2)) return false;
  res = big_cmp(l, r);
  if (res == 0 && sticky) res = 1;
  return true;
}

// JSON.parse's value of the number text [p, e) (already validated: -?int(.frac)?(e[+-]?exp)?).
// false: the digits overflowed a limb bound (not reachable for inputs under 2^32 bytes; refused).
YC_HD inline bool dec_to_f64(const uint8_t* __restrict__ b, uint32_t p, uint32_t e, double& out) {
  const bool neg = b[p] == '-';
  if (neg) ++p;
  BigD D;
  D.n = 0;
  uint32_t kept = 0;
  bool sticky = false, lead = true;
  int64_t dot = 0;       // decimal exponent of the last kept digit's position, before the exponent part
  uint32_t chunk = 0, cn = 0;
  bool in_frac = false;
  uint32_t q = p;
  for (; q < e; ++q) {
    const uint32_t c = b[q];
    if (c == '.') { in_frac = true; continue; }
    if (c < '0' || c > '9') break;
    if (lead && c == '0') { if (in_frac) --dot; continue; }
    lead = false;
    if (kept < DEC_MAX_DIGITS) {
      chunk = chunk * 10 + (c - '0');
      if (++cn == 9) {
        if (!big_mul_small(D, 1000000000u, chunk)) return false;
        chunk = 0;
        cn = 0;
      }
      ++kept;
      if (in_frac) --dot;
    } else {
      if (c != '0') sticky = true;
      if (!in_frac) ++dot;
    }
  }
  if (cn) {
    uint32_t pw = 1;
    for (uint32_t i = 0; i < cn; ++i) pw *= 10;
    if (!big_mul_small(D, pw, chunk)) return false;
  }
  int64_t ex = 0;
  if (q < e && (b[q] == 'e' || b[q] == 'E')) {
    ++q;
    bool en = false;
    if (q < e && (b[q] == '+' || b[q] == '-')) { en = b[q] == '-'; ++q; }
    for (; q < e && b[q] >= '0' && b[q] <= '9'; ++q)
      if (ex < 100000000) ex = ex * 10 + (b[q] - '0');
    if (en) ex = -ex;
  }
  if (kept == 0) { out = neg ? -0.0 : 0.0; return true; }
  const int64_t E64 = dot + ex;                   // value = D * 10^E (+ sticky)
  const int64_t n10 = E64 + (int64_t)kept;        // value = 0.d1d2.. * 10^n10
  if (n10 > 310) { out = f64_from(neg ? 0xFFF0000000000000ull : 0x7FF0000000000000ull); return true; }
  if (n10 < -324) { out = neg ? -0.0 : 0.0; return true; }  // below 10^-324 < half the least subnormal
  const int32_t E = (int32_t)E64;
  // a first guess from the leading 19 digits (within a few ulps), then exact midpoint tests
  uint64_t top = 0;
  uint32_t tk = 0;
  {
    bool ld = true;
    for (uint32_t r = p; r < e && tk < 19; ++r) {
      const uint32_t c = b[r];
      if (c == '.') continue;
      if (c < '0' || c > '9') break;
      if (ld && c == '0') continue;
      ld = false;
      top = top * 10 + (c - '0');
      ++tk;
    }
  }
  double x = (double)top;
  int32_t s10 = (int32_t)(n10 - (int64_t)tk);  // x * 10^s10 ~ value
  // scale in steps that keep x normal: divide last only after multiplying up
  while (s10 > 0) { const int32_t k = s10 > 22 ? 22 : s10; double f = 1; for (int32_t i = 0; i < k; ++i) f *= 10; x *= f; s10 -= k; }
  while (s10 < 0) { const int32_t k = s10 < -22 ? 22 : -s10; double f = 1; for (int32_t i = 0; i < k; ++i) f *= 10; x /= f; s10 += k; }
  uint64_t bits = f64_bits(x);
  if ((bits >> 52) >= 0x7FFu) bits = 0x7FEFFFFFFFFFFFFFull;  // past the largest finite: start there
  if (bits == 0) bits = 1;                                    // below the least subnormal: start there
  BigD l, r;
  for (int it = 0; it < 4096; ++it) {
    uint64_t m;
    int32_t qq;
    f64_split(bits, m, qq);
    int c;
    if (!dec_cmp_mid(D, E, sticky, m, qq, l, r, c)) return false;
    if (c > 0 || (c == 0 && (bits & 1u))) {  // above the midpoint with the next double (a tie: the even one)
      ++bits;
      if ((bits >> 52) >= 0x7FFu) { out = f64_from(neg ? 0xFFF0000000000000ull : 0x7FF0000000000000ull); return true; }
      continue;
    }
    if (bits == 0) break;
    f64_split(bits - 1, m, qq);
    if (!dec_cmp_mid(D, E, sticky, m, qq, l, r, c)) return false;
    if (c < 0 || (c == 0 && (bits & 1u))) { --bits; continue; }  // below the midpoint with the previous one
    break;
  }
  out = f64_from(bits | (neg ? 1ull << 63 : 0ull));
  return true;
}

// Number::toString's digits of a finite double x > 0: d[0..k) and the decimal point position n
// (x ~ 0.d1d2..dk * 10^n). k <= 17.
constexpr int SHORT_LIMBS = 40;  // 1 280 bits: 2^1077 and 10^324 scales
using BigS = BigN<SHORT_LIMBS>;
YC_HD inline uint32_t f64_shortest(double x, char* d, int32_t& n) {
  uint64_t m;
  int32_t e;
  f64_split(f64_bits(x), m, e);
  const bool even = (m & 1u) == 0;
  const bool lower_closer = m == (1ull << 52) && e > -1074;  // the gap below is half the gap above
  BigS R, S, Mp, Mm, T;
  // x = R / S; the rounding interval is (x - Mm/S, x + Mp/S), both bounds kept for an even m
  if (e >= 0) {
    big_set(R, m);
    big_shl(R, (uint32_t)e + (lower_closer ? 2u : 1u));
    big_set(S, lower_closer ? 4u : 2u);
    big_set(Mp, 1);
    big_shl(Mp, (uint32_t)e + (lower_closer ? 1u : 0u));
    big_set(Mm, 1);
    big_shl(Mm, (uint32_t)e);
  } else {
    big_set(R, m);
    big_shl(R, lower_closer ? 2u : 1u);
    big_set(S, 1);
    big_shl(S, (uint32_t)(-e) + (lower_closer ? 2u : 1u));
    big_set(Mp, lower_closer ? 2u : 1u);
    big_set(Mm, 1);
  }
  // k ~ ceil(log10(x)): an estimate from the binary exponent, corrected below
  int32_t bl = 0;
  for (uint64_t t = m; t; t >>= 1) ++bl;
  const double lg = (double)(e + bl - 1) * 0.30102999566398114;
  int32_t k = (int32_t)lg;
  if ((double)k < lg) ++k;  // ceil
  if (k >= 0) {
    for (int32_t i = 0; i < k; ++i) big_mul_small(S, 10);
  } else {
    for (int32_t i = 0; i < -k; ++i) { big_mul_small(R, 10); big_mul_small(Mp, 10); big_mul_small(Mm, 10); }
  }
  // fix the estimate: the first digit must be nonzero and (R + Mp) / S < 1 (<= for an even m)
  for (;;) {
    const int c = big_plus_cmp(R, Mp, S, T);
    if (c > 0 || (even && c == 0)) { big_mul_small(S, 10); ++k; continue; }
    break;
  }
  for (;;) {
    // (R + Mp) * 10 / S >= 1 is where the first digit is nonzero
    BigS R10 = R, Mp10 = Mp;
    big_mul_small(R10, 10);
    big_mul_small(Mp10, 10);
    const int c = big_plus_cmp(R10, Mp10, S, T);
    if (c < 0 || (!even && c == 0)) { R = R10; Mp = Mp10; big_mul_small(Mm, 10); --k; continue; }
    break;
  }
  n = k;
  uint32_t nd = 0;
  for (;;) {
    big_mul_small(R, 10);
    big_mul_small(Mp, 10);
    big_mul_small(Mm, 10);
    uint32_t digit = 0;
    while (big_cmp(R, S) >= 0) { big_sub(R, S); ++digit; }
    const int cl = big_cmp(R, Mm);
    const bool low = even ? cl <= 0 : cl < 0;
    const int ch = big_plus_cmp(R, Mp, S, T);
    const bool high = even ? ch >= 0 : ch > 0;
    if (!low && !high && nd < 17) { d[nd++] = (char)('0' + digit); continue; }
    if (low && high) {  // both neighbours qualify: the nearer one (2R vs S); a tie takes the even digit
      T = R;
      big_shl(T, 1);
      const int c2 = big_cmp(T, S);
      if (c2 > 0 || (c2 == 0 && (digit & 1u))) ++digit;
    } else if (high) {
      ++digit;
    }
    d[nd++] = (char)('0' + digit);
    break;
  }
  return nd;
}

// Number::toString's text (radix 10) of digits d[0..k) with point position n; t holds >= 32 bytes
YC_HD inline uint32_t num_text(bool neg, const char* d, uint32_t k, int32_t n, char* t) {
  uint32_t m = 0;
  if (k == 0) { t[m++] = '0'; return m; }  // (-0 is written "0")
  if (neg) t[m++] = '-';
  if ((int32_t)k <= n && n <= 21) {
    for (uint32_t i = 0; i < k; ++i) t[m++] = d[i];
    for (int32_t i = (int32_t)k; i < n; ++i) t[m++] = '0';
  } else if (0 < n && n <= 21) {
    for (int32_t i = 0; i < n; ++i) t[m++] = d[i];
    t[m++] = '.';
    for (uint32_t i = (uint32_t)n; i < k; ++i) t[m++] = d[i];
  } else if (-6 < n && n <= 0) {
    t[m++] = '0';
    t[m++] = '.';
    for (int32_t i = 0; i < -n; ++i) t[m++] = '0';
    for (uint32_t i = 0; i < k; ++i) t[m++] = d[i];
  } else {
    t[m++] = d[0];
    if (k > 1) { t[m++] = '.'; for (uint32_t i = 1; i < k; ++i) t[m++] = d[i]; }
    t[m++] = 'e';
    int32_t x = n - 1;
    t[m++] = x < 0 ? '-' : '+';
    if (x < 0) x = -x;
    char r[4];
    uint32_t nr = 0;
    do { r[nr++] = (char)('0' + x % 10); x /= 10; } while (x);
    while (nr) t[m++] = r[--nr];
  }
  return m;
}

// JSON.stringify(JSON.parse(number text [p, e))) into t (>= 32 bytes): its length, 0 when the
// digits overflow the limb bounds. An infinity is written "null", as JSON.stringify writes it.
YC_HD inline __attribute__((noinline)) uint32_t json_number_canon(const uint8_t* __restrict__ b, uint32_t p, uint32_t e, char* t) {
  double x;
  if (!dec_to_f64(b, p, e, x)) return 0;
  const uint64_t bits = f64_bits(x);
  if (((bits >> 52) & 0x7FFu) == 0x7FFu) { t[0] = 'n'; t[1] = 'u'; t[2] = 'l'; t[3] = 'l'; return 4; }
  if ((bits << 1) == 0) { t[0] = '0'; return 1; }
  char d[20];
  int32_t n;
  const uint32_t k = f64_shortest(f64_from(bits & ~(1ull << 63)), d, n);
  return num_text((bits >> 63) != 0, d, k, n, t);
}

}  // namespace yc
