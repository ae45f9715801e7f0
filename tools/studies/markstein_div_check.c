/* Study: the quotient RN(x/d) from a precomputed y = RN(1/d) by one Markstein correction
 *   q0 = RN(x*y); r = fma(-q0, d, x); q = fma(r, y, q0)
 * compared with the IEEE division, bit for bit, over random and adversarial operands in the range
 * the learned-grid kernels take the fast path for (|d| in [2^-100, 2^100], x != 0,
 * |q| in [2^-100, 2^100]). Build: gcc -O2 -o /tmp/mk markstein_div_check.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static int check(float x, float d, float y, long* fast, long* bad)
{
    volatile float q0 = x * y;
    float r = fmaf(-q0, d, x);
    float q = fmaf(r, y, q0);
    float aq = fabsf(q);
    float ax = fabsf(x);
    if (!(ax >= 0x1p-100f && ax <= 0x1p100f && aq >= 0x1p-100f && aq <= 0x1p100f))
        return 0;
    ++*fast;
    float want = x / d;
    if (u_of(q) != u_of(want)) {
        if (*bad < 10) printf("MISMATCH x=%a d=%a q=%a want=%a\n", x, d, q, want);
        ++*bad;
        return 1;
    }
    return 0;
}

int main(void)
{
    long fast = 0, bad = 0;
    for (int k = 0; k < 4000; ++k) {
        /* d: random normal float in [2^-100, 2^100], plus mantissas near all-ones / powers of two */
        uint32_t e = 27 + (uint32_t)(rnd() % 200), m = (uint32_t)(rnd() & 0x7FFFFF);
        if (k % 7 == 0) m = 0x7FFFFF - (uint32_t)(rnd() % 16);
        if (k % 11 == 0) m = (uint32_t)(rnd() % 16);
        float d = f_of((e << 23) | m);
        if (k & 1) d = -d;
        float y = 1.0f / d;
        for (int j = 0; j < 250000; ++j) {
            float x;
            uint64_t t = rnd();
            if (j % 4 == 0) {
                /* near half-integer quotients: x = (n + 0.5 +- tiny) * d */
                float n = (float)((int64_t)(t % 140000) - 70000);
                x = (n + 0.5f) * d;
                x = f_of(u_of(x) + (int32_t)((t >> 40) % 7) - 3);
            } else if (j % 4 == 1) {
                /* quotients in [-2^17, 2^17] */
                x = (float)((double)((int64_t)(t % (1u << 30)) - (1 << 29)) / 4096.0) * d;
            } else {
                x = f_of((uint32_t)(t & 0xFFFFFFFF));
                if (!isfinite(x)) continue;
            }
            check(x, d, y, &fast, &bad);
        }
    }
    printf("checked %ld fast-path quotients, %ld mismatches\n", fast, bad);
    return bad != 0;
}
