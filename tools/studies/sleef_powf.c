/* Study: the C form of the device Sleef powf_u10 restatement (aimet_amd/csrc/adaround.hip: pow01),
 * checked against torch.pow on the CPU by tools/studies/sleef_powf_check.py. */
#include <math.h>
#include <stdint.h>
#include <string.h>
typedef struct { float x, y; } f2;
static inline float fmapn(float x, float y, float z) { return fmaf(x, y, -z); }
static inline float fmanp(float x, float y, float z) { return fmaf(-x, y, z); }
static inline f2 mk(float x, float y) { f2 r = {x, y}; return r; }
static inline f2 dfnormalize(f2 t) { float s = t.x + t.y; return mk(s, (t.x - s) + t.y); }
static inline f2 dfscale(f2 d, float s) { return mk(d.x * s, d.y * s); }
static inline f2 dfadd2_ff(float x, float y) { float s = x + y; float v = s - x; return mk(s, (x - (s - v)) + (y - v)); }
static inline f2 dfadd2_f2f(f2 x, float y) { float s = x.x + y; float v = s - x.x; float t = (x.x - (s - v)) + (y - v); return mk(s, t + x.y); }
static inline f2 dfadd_f2f2(f2 x, f2 y) { float s = x.x + y.x; return mk(s, (((x.x - s) + y.x) + x.y) + y.y); }
static inline f2 dfadd2_f2f2(f2 x, f2 y) { float s = x.x + y.x; float v = s - x.x; float t = (x.x - (s - v)) + (y.x - v); return mk(s, t + (x.y + y.y)); }
static inline f2 dfadd_ff2(float x, f2 y) { float s = x + y.x; return mk(s, ((x - s) + y.x) + y.y); }
static inline f2 dfmul_ff(float x, float y) { float s = x * y; return mk(s, fmapn(x, y, s)); }
static inline f2 dfsqu(f2 x) { float s = x.x * x.x; return mk(s, fmaf(x.x + x.x, x.y, fmapn(x.x, x.x, s))); }
static inline f2 dfmul_f2f2(f2 x, f2 y) { float s = x.x * y.x; return mk(s, fmaf(x.x, y.y, fmaf(x.y, y.x, fmapn(x.x, y.x, s)))); }
static inline f2 dfmul_f2f(f2 x, float y) { float s = x.x * y; return mk(s, fmaf(x.y, y, fmapn(x.x, y, s))); }
static inline f2 dfdiv(f2 n, f2 d) {
  float t = 1.0f / d.x; float s = n.x * t; float u = fmapn(t, n.x, s);
  float v = fmanp(d.y, t, fmanp(d.x, t, 1.0f));
  return mk(s, fmaf(s, v, fmaf(n.y, t, u)));
}
static inline float as_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t as_u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
/* AVX512 getexp: floor(log2|x|) as float (x normal) */
static inline float getexp(float x) { int e; frexpf(x, &e); return (float)(e - 1); }
/* AVX512 getmant, interval [0.75, 1.5) */
static inline float getmant_p75(float x) {
  int e; float m = frexpf(fabsf(x), &e);   /* m in [0.5, 1) */
  m = m * 2.0f;                            /* [1, 2) */
  if (m >= 1.5f) m = m * 0.5f;             /* [0.75, 1.5) */
  return m;
}
static f2 logkf(float d) {
  float e = getexp(d * (1.0f / 0.75f));
  if (isinf(e) && e > 0) e = 128.0f;
  float m = getmant_p75(d);
  f2 x = dfdiv(dfadd2_ff(-1.0f, m), dfadd2_ff(1.0f, m));
  f2 x2 = dfsqu(x);
  float t = 0.240320354700088500976562f;
  t = fmaf(t, x2.x, 0.285112679004669189453125f);
  t = fmaf(t, x2.x, 0.400007992982864379882812f);
  f2 c = mk(0.66666662693023681640625f, 3.69183861259614332084311e-09f);
  f2 s = dfmul_f2f(mk(0.69314718246459960938f, -1.904654323148236017e-09f), e);
  s = dfadd_f2f2(s, dfscale(x, 2.0f));
  s = dfadd_f2f2(s, dfmul_f2f2(dfmul_f2f2(x2, x), dfadd2_f2f2(dfmul_f2f(x2, t), c)));
  return s;
}
static float vldexp(float x, int q) {
  int m = q >> 31;
  m = (((m + q) >> 6) - m) << 4;
  q = q - (m << 2);
  m = 0x7f + m;
  m = (0 > m) ? 0 : m;
  m = (m > 0xff) ? 0xff : m;
  float u = as_f((uint32_t)m << 23);
  x = x * u * u * u * u;
  u = as_f((uint32_t)(q + 0x7f) << 23);
  return x * u;
}
static float expkf(f2 d) {
  float u = (d.x + d.y) * 1.442695040888963407359924681001892137426645954152985934135449406931f;
  int q = (int)rintf(u);
  f2 s, t;
  s = dfadd2_f2f(d, (float)q * -0.693145751953125f);
  s = dfadd2_f2f(s, (float)q * -1.428606765330187045e-06f);
  s = dfnormalize(s);
  u = 0.00136324646882712841033936f;
  u = fmaf(u, s.x, 0.00836596917361021041870117f);
  u = fmaf(u, s.x, 0.0416710823774337768554688f);
  u = fmaf(u, s.x, 0.166665524244308471679688f);
  u = fmaf(u, s.x, 0.499999850988388061523438f);
  t = dfadd_f2f2(s, dfmul_f2f(dfsqu(s), u));
  t = dfadd_ff2(1.0f, t);
  u = t.x + t.y;
  u = vldexp(u, q);
  if (d.x < -104.0f) u = 0.0f;
  return u;
}
/* powf for x >= 0 finite, y finite (the AdaRound case) */
float sleef_powf_u10(float x, float y) {
  float result = expkf(dfmul_f2f(logkf(fabsf(x)), y));
  if (isnan(result)) result = INFINITY;
  result = result * (x > 0 ? 1.0f : NAN);  /* x < 0 handled below only for completeness */
  if (x == 0.0f) result = (signbit(y) ? INFINITY : 0.0f);
  if (y == 0.0f || x == 1.0f) result = 1.0f;
  return result;
}
void sleef_powf_arr(const float* x, float y, float* out, long n) { for (long i = 0; i < n; ++i) out[i] = sleef_powf_u10(x[i], y); }
