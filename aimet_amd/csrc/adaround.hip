// adaround.hip -- fused AdaRound soft-quantization forward and backward for gfx950.
//
// Reference (pure torch, ~6 elementwise kernels forward and ~10 backward per iteration, each a
// full pass over the weight): AdaroundWrapper.apply_adaround (v1/adaround/adaround_wrapper.py:124-149)
// and AdaroundLoss.compute_round_loss (v1/adaround/adaround_loss.py:83-110), ZETA = 1.1,
// GAMMA = -0.1 (aimet_common/defs.py:302-306).
//
// Here: one pass forward (reads W, alpha; writes Wq: 12 B/elem) and one pass backward (reads
// grad_Wq, W, alpha; writes grad_alpha: 16 B/elem) that also produces the rounding-loss term
// and its gradient.
//
// Numerics: the reference's arithmetic is torch float32 ops on the CPU; every op here is the same
// IEEE operation in the same order, and the sigmoid is torch's own vectorized CPU sigmoid
// (1 / (1 + expf(-a)) with Sleef's expf_u10 polynomial, FMA form, then an IEEE divide), so Wq is
// bit-identical to the reference (tests/golden/golden_adaround.npz). The rounding loss's
// pow(|2h-1|, beta) / pow(|2h-1|, beta-1) is, by default, the table-driven f32 pow of
// fast_pow.hpp: within 1 ulp of torch's CPU pow (Sleef powf_u10) for every f32 |2h-1| in (0, 1)
// and every exponent of the AdaRound schedules (profiles/r06/pow_fast_check.txt), at ~33 f32
// instructions and 2 LDS reads instead of Sleef's ~142 f32 instructions. aimet_adaround_set_exact_pow(1) selects the bit-exact emulation of
// torch's pow instead (sleef_pow.hpp: Sleef powf_u10 in the vectorized part, the scalar tail as
// std::pow), with which dL/dalpha, the rounding-loss term included, is bit-identical too.
#include "common.hpp"
#include "fast_pow.hpp"
#include "recon.hpp"
#include "sleef_pow.hpp"

#include <atomic>

namespace aimet_amd
{
namespace
{

constexpr float kGamma = -0.1f;
// python: (ZETA - GAMMA) = 1.2000000000000002 -> float32 scalar 1.2f in the torch op
constexpr float kZmG = (float) (1.1 - (-0.1));
constexpr int kAdaBwdGrid = 8192;   // 32 workgroups per CU; bounds the round-loss partials
#ifndef AIMET_ADA_BWD_U
#define AIMET_ADA_BWD_U 1   // quads per lane per tile of adaround_bwd_vec_kernel
#endif

struct AdaChannel
{
    FastDiv divK, divC;
    uint32_t C;
    __device__ __forceinline__ uint32_t channel(uint32_t i) const
    {
        if (C == 1)
            return 0;
        uint32_t row = divK.div(i);
        return row - divC.div(row) * C;
    }
};

typedef float f4 __attribute__((ext_vector_type(4)));

// expf as torch's CPU vector code computes it (ATen Vectorized<float>::exp = Sleef expf_u10):
// q = rint(d * log2(e)); s = d - q*ln2 in two FMA steps (Cody-Waite); a degree-6 polynomial in
// Horner FMA form; 2^q applied; d < -104 -> 0, d > 100 -> inf. Every step is an IEEE op, so the
// result is Sleef's bit for bit wherever it is normal. A correctly rounded expf would differ from
// it in ~1% of inputs and the difference reaches Wq unattenuated where floor(W/delta) + h - offset
// nearly cancels. Sleef applies 2^q as two power-of-two multiplies (vldexp2); one v_ldexp_f32 is
// the same exact scaling except where the result is subnormal (d < -87.3), which only feeds
// sigmoidf's e + 1 == 1 (tools/studies/sigmoid_fast_check.hip: all 2^32 sigmoid inputs equal).
__device__ __forceinline__ float sigmoid_expf(float d)
{
    const float qf = __builtin_rintf(d * 1.442695040888963407359924681001892137426645954152985934135449406931f);
    const int q    = (int) qf;
    float s        = __builtin_fmaf(qf, -0.693145751953125f, d);
    s              = __builtin_fmaf(qf, -1.428606765330187045e-06f, s);
    float u        = 0.000198527617612853646278381f;
    u              = __builtin_fmaf(u, s, 0.00139304355252534151077271f);
    u              = __builtin_fmaf(u, s, 0.00833336077630519866943359f);
    u              = __builtin_fmaf(u, s, 0.0416664853692054748535156f);
    u              = __builtin_fmaf(u, s, 0.166666671633720397949219f);
    u              = __builtin_fmaf(u, s, 0.5f);
    u              = __builtin_ldexpf(1.0f + __builtin_fmaf(s * s, u, s), q);
    u              = d < -104.0f ? 0.0f : u;
    return d > 100.0f ? __builtin_inff() : u;
}

// torch.clamp(x, lo, hi) on the CPU (vectorized kernel: NaN propagates; maximum / minimum are
// x86 MAXPS / MINPS, which return the second operand unless the first is strictly greater / less,
// so clamp(-0.0, 0, 1) is +0.0)
__device__ __forceinline__ float clamp_torch(float x, float lo, float hi)
{
    if (x != x)
        return x;
    const float m = x > lo ? x : lo;
    return m < hi ? m : hi;
}

// torch.sigmoid on the CPU (vectorized kernel): a = 0 - a; a = exp(a); a = a + 1; 1 / a. The IEEE
// division 1 / y as v_rcp_f32 + one Newton step: equal to it for every y in [1, 2^126), the range
// of e + 1 here below 2^126 (tools/studies/sigmoid_fast_check.hip, exhaustive); beyond, the division.
__device__ __forceinline__ float sigmoidf(float a)
{
    // -a for 0 - a: they differ only at a = +0 (-0 against +0), and sigmoid_expf(+-0) is 1 either
    // way (every use of its argument is a product, a sum with a signed-zero-insensitive result or a
    // comparison); the negation folds into the first instructions' source modifiers
    const float y = sigmoid_expf(-a) + 1.0f;
    if (y < 0x1p126f)
    {
        const float r = __builtin_amdgcn_rcpf(y);
        return __builtin_fmaf(__builtin_fmaf(-y, r, 1.0f), r, r);
    }
    return 1.0f / y;
}

// floor(w / d) exactly as the IEEE division gives it, from q = w * rcp (rcp = v_rcp_f32(d), within
// 1 ulp): |q - RN(w/d)| <= 3.5 ulp(q) < 2^-21 (|q| + 1), so when q lies farther than that from
// every integer both floors agree; otherwise (and for non-finite q) the division decides.
// The distances to floor(q) and floor(q) + 1 as fr = v_fract_f32(q) and 1 - fr: each within 2^-24
// of the exact distance (fr < 1 after its rounding, clamped to 1 - 2^-24 where it would round to
// 1), and the threshold exceeds the quotient's 3.5 ulp by at least 2^-21, so a margin above it
// still proves the floors equal. Either branch returns floor(w / d): the guard only picks how.
__device__ __forceinline__ float floor_div(float w, float d, float rcp)
{
    const float q   = w * rcp;
    const float f   = __builtin_floorf(q);
    const float fr  = __builtin_amdgcn_fractf(q);
    // (|q| + 1) 2^-21 in one instruction: scaling by a power of two commutes with the rounding
    const float thr = __builtin_fmaf(__builtin_fabsf(q), 4.76837158203125e-7f, 4.76837158203125e-7f);
    if (fr > thr && 1.0f - fr > thr)
        return f;
    return __builtin_floorf(w / d);
}

struct AdaParams
{
    float qmax, reg, beta, beta_m1;   // beta_m1 = (float)(beta - 1) in double, as torch's pow_backward
    int soft;
    uint32_t vec_end;   // n - n % 32: the reference's pow runs elements >= vec_end in its scalar tail
    int want_loss;      // the rounding-loss value is requested (else only its gradient's pow runs)
};

__device__ __forceinline__ float ada_fwd(float w, float a, float d, float o, const AdaParams& p, float rcp)
{
    float t = floor_div(w, d, rcp);   // == floor of the IEEE division (floor is sensitive to the last ulp)
    float h;
    if (p.soft)
    {
        float pre = sigmoidf(a) * kZmG + kGamma;
        h         = clamp_torch(pre, 0.0f, 1.0f);
    }
    else
        h = a >= 0.0f ? 1.0f : 0.0f;
    float q = clamp_torch(t + h - o, 0.0f, p.qmax);
    return (q + o) * d;
}

// dL/dalpha of Wq without the rounding loss (clamp pass-through masks as torch autograd); also
// returns what the rounding-loss terms need: sigmoid(alpha), x = 2h - 1 and whether h lies inside
// its clamp (in_h). Outside it h is exactly 0 or 1, so |x| = 1 (or NaN) and the loss's pow needs
// no logarithm.
__device__ __forceinline__ float ada_bwd_base(float w, float a, float g, float d, float o, const AdaParams& p,
                                              float rcp, float& sg, float& x, bool& in_h)
{
    float t   = floor_div(w, d, rcp);
    sg        = sigmoidf(a);
    float pre = sg * kZmG + kGamma;
    // clamp_torch(pre, 0, 1) as v_max / v_min, NaN restored after (they return the other operand):
    // pre is never -0 (a sum with -0.1f is -0 only for -0 operands), so the two forms agree
    float h   = __builtin_fminf(__builtin_fmaxf(pre, 0.0f), 1.0f);
    h         = pre != pre ? pre : h;
    float u   = t + h - o;
    // autograd of apply_adaround, op by op: d wq / d tq = g * delta; clamp_backward passes it where
    // min <= x <= max; the adds pass it on; h's clamp likewise; mul by (zeta - gamma) -> * 1.2f;
    // sigmoid_backward: (grad * (1 - s)) * s. pre lies in [0, 1] exactly where the clamp returns it
    // (a NaN pre compares unequal)
    in_h     = h == pre;
    float gh = (u >= 0.0f && u <= p.qmax) ? g * d : 0.0f;
    x        = __builtin_fmaf(2.0f, h, -1.0f);   // 2h is exact: one rounding, as 2.0f * h + -1.0f
    return ((in_h ? gh : 0.0f) * kZmG * (1.0f - sg)) * sg;
}

// the rounding loss's pow terms need Sleef's logkf only for |x| in (0, 1) outside the scalar tail
// (pow01_log's other cases are exact constants, products or the tail's double pow)
__device__ __forceinline__ bool ada_needs_log(float ax, bool tail)
{
    return !(ax == 0.0f || ax == 1.0f || tail);
}

// compute_round_loss's own graph (adaround_loss.py:97-110), summed into alpha's gradient as
// autograd does: round_loss = reg * sum(1 - |2h - 1|^beta); grad -reg at the pow; pow_backward:
// grad * (beta * x^(beta - 1)) (= pbm1 here); abs: * sgn(x); 2*h: * 2. Lanes outside h's clamp add
// the selected +0 term as the full expression does.
// SIGN_FAST (the caller checks reg > 0, beta > 0 and beta - 1 > 0, uniformly): then dpw <= 0, and
// on lanes inside h's clamp (the only ones whose dh is used) x = 2h - 1 is finite and never -0, and
// at x = +0 the pow is 0 so dpw = -0; (dpw * sgn(x)) * 2 is then -copysign(2 dpw, x) exactly
template <bool SIGN_FAST = false>
__device__ __forceinline__ float ada_bwd_round(float ga, float sg, float x, bool in_h, float pbm1, const AdaParams& p)
{
    float dh;
    if constexpr (SIGN_FAST)   // -(reg (beta p)) is (-reg) (beta p) exactly: the negations go last
        dh = -__builtin_copysignf((p.reg * (p.beta * pbm1)) * 2.0f, x);
    else
    {
        float dpw = (-p.reg) * (p.beta * pbm1);
        dh        = (dpw * (x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f))) * 2.0f;
    }
    return ga + ((in_h ? dh : 0.0f) * kZmG * (1.0f - sg)) * sg;
}

// dL/dalpha of Wq + the rounding-loss gradient, one element (the loss term added to `loss`).
// EXACT: the rounding loss's pow is the bit-exact emulation of torch's (sleef_pow.hpp), else the
// fast pow (fast_pow.hpp, within 1 ulp of it; its tables filled into LDS by the kernel)
template <bool EXACT>
__device__ __forceinline__ float ada_bwd(float w, float a, float g, float d, float o, const AdaParams& p, float rcp,
                                         float& loss, uint32_t idx)
{
    float sg, x;
    bool in_h;
    float ga = ada_bwd_base(w, a, g, d, o, p, rcp, sg, x, in_h);
    if (p.reg != 0.0f)
    {
        const bool tail = idx >= p.vec_end;
        const float ax  = fabsf(x);
        float pbm1      = 0.0f;
        // only lanes inside h's clamp use the gradient's pow, and the logarithm only where it is not
        // an exact case: a real branch, so a wave whose alphas all saturate skips the logarithm and
        // the exponentials (the skipped values were dead: the selects below drop them)
        if (in_h || p.want_loss)
        {
            if constexpr (EXACT)
            {
                F2 l {0.0f, 0.0f};
                if (ada_needs_log(ax, tail))
                    l = sleef_logkf(ax);
                if (p.want_loss)
                    loss += 1.0f - pow01_log(ax, p.beta, tail, l);
                if (in_h)
                    pbm1 = pow01_log(ax, p.beta_m1, tail, l);
            }
            else
            {
                LnSplit l {0.0f, 0.0f};
                if (!(ax == 0.0f || ax == 1.0f))
                    l = ln01(ax);
                if (p.want_loss)
                    loss += 1.0f - pow01_fast_l(ax, p.beta, l);
                if (in_h)
                    pbm1 = pow01_fast_l(ax, p.beta_m1, l);
            }
        }
        ga = ada_bwd_round(ga, sg, x, in_h, pbm1, p);
    }
    return ga;
}

// pow01_log for |x| in {0, 1} (its exact early returns, whatever the exponent)
__device__ __forceinline__ float pow01_exact(float ax, float e)
{
    return ax == 0.0f ? (e == 0.0f ? 1.0f : 0.0f) : 1.0f;
}

// E elements per lane whose rounding-loss pow terms are evaluated wave-compacted: every used
// element (inside h's clamp, or any element when the loss is requested) whose |x| is not 0 or 1
// -- the ones that need Sleef's logkf, or the scalar tail's double pow -- is packed densely into
// this wave's LDS slot (ballot + mbcnt prefix; the tail ones stored negated), evaluated
// ceil(count / 64) per lane, and read back. A wave then pays for the logarithm in proportion to
// the elements that need it, not to the elements any of its lanes hold (saturated alphas in a
// converging AdaRound loop are mixed with unsaturated ones in every wave). Every value is the
// same function of |x| as pow01_log's, so the results are bit-identical to ada_bwd. The slot is
// the wave's own, so the lanes only order their LDS accesses among themselves (wave_sync); the
// wave's lanes must all call it. `wl` = 2 * 64 * E floats per wave. TAIL = false
// when no element of the wave's tile lies in the scalar tail (every tile but the last): the tail
// flags are then compile-time false and cost nothing per element.
// the LDS writes of this wave's lanes visible to its other lanes (a wave's LDS operations complete
// in order; the fences keep the compiler from moving accesses across)
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int E, bool TAIL, bool EXACT>
__device__ __forceinline__ void ada_round_pows(const float (&ax)[E], const bool (&tail_in)[E], const bool (&use)[E],
                                               const AdaParams& p, float* __restrict__ wl, float (&pbm1)[E],
                                               float (&pb)[E])
{
    const uint32_t lane = threadIdx.x & 63;
    bool need[E], tail[E];
    uint64_t ballot[E];   // the lane masks themselves (__ballot would round-trip each flag through a VGPR)
    auto find_need = [&]() {
#pragma unroll
        for (int k = 0; k < E; ++k)
        {
            need[k]   = use[k] && !(ax[k] == 0.0f || ax[k] == 1.0f);
            ballot[k] = __builtin_amdgcn_ballot_w64(need[k]);
        }
    };
    // the dense test counts the elements with |x| < 1 (inside h's clamp, give or take the rare
    // |x| = 0 or an h clamped exactly at 0 or 1): it only picks between forms with the same values,
    // and the ballot of one comparison is that comparison's lane mask (no VGPR round trip)
    uint32_t total = 0;
#pragma unroll
    for (int k = 0; k < E; ++k)
    {
        tail[k] = TAIL && tail_in[k];
        total += (uint32_t) __popcll(__builtin_amdgcn_ballot_w64(ax[k] < 1.0f));
    }
    if (!EXACT && 4 * total >= 3 * 64 * E)
    {
        // a dense wave: each lane evaluates its own elements in place with the fast pow (its
        // logarithm shared by the two exponents; the scalar tail takes it too: fast_pow.hpp).
        // Exponents other than 0, 2, 3 (uniform): branch-free -- every element is evaluated (on a
        // stand-in 0.5 where |x| is 0 or 1) and the exact cases selected after, so the wave keeps
        // no per-element exec masks (the pow runs for most lanes of a dense wave anyway)
        const bool generic_m1 = !(p.beta_m1 == 0.0f || p.beta_m1 == 2.0f || p.beta_m1 == 3.0f);
        const bool generic_b  = !(p.beta == 0.0f || p.beta == 2.0f || p.beta == 3.0f);
        if (generic_m1 && (!p.want_loss || generic_b))
        {
#pragma unroll
            for (int k = 0; k < E; ++k)
            {
                // |x| outside (0, 1) is 0, 1 or NaN (x = 2h - 1, h clamped to [0, 1]): pow01_fast_l's
                // exact cases give 0, 1 and, for NaN, inf -- |x| itself, or inf for NaN. ln01 and
                // exp_ln run on those too (every step stays in range: table indices are masked, a
                // NaN converts to n = 0) and their value is dropped
                const bool inside = ax[k] > 0.0f && ax[k] < 1.0f;
                const LnSplit l   = ln01(ax[k]);
                const float fixed = ax[k] != ax[k] ? __builtin_inff() : ax[k];
                pbm1[k]           = inside ? exp_ln(l, p.beta_m1) : fixed;
                pb[k]             = p.want_loss ? (inside ? exp_ln(l, p.beta) : fixed) : 0.0f;
            }
            return;
        }
        find_need();
#pragma unroll
        for (int k = 0; k < E; ++k)
        {
            if (need[k])
            {
                const LnSplit l = ln01(ax[k]);
                pbm1[k]        = pow01_fast_l(ax[k], p.beta_m1, l);
                pb[k]          = p.want_loss ? pow01_fast_l(ax[k], p.beta, l) : 0.0f;
            }
            else
            {
                pbm1[k] = pow01_exact(ax[k], p.beta_m1);
                pb[k]   = pow01_exact(ax[k], p.beta);
            }
        }
        return;
    }
    find_need();
    if (EXACT && 4 * total >= 3 * 64 * E)
    {
        // a dense wave (few saturated alphas): each lane evaluates its own elements in place, the
        // compaction's LDS round trip would not pay (the same values), two at a time in packed f32
        // (vsleef_logkf / vpow01_log: component by component the scalar arithmetic). A pair with no
        // element needing the logarithm skips it; an element that does not need it takes its exact
        // value (its packed component is computed on a harmless stand-in, 0.5, and dropped).
#pragma unroll
        for (int k = 0; k + 1 < E; k += 2)
        {
            if (need[k] || need[k + 1])
            {
                const fl2 xv {need[k] ? ax[k] : 0.5f, need[k + 1] ? ax[k + 1] : 0.5f};
                V2 l {vsplat(0.0f), vsplat(0.0f)};
                if (!(tail[k] && tail[k + 1]))
                    l = vsleef_logkf(xv);
                const fl2 r1 = vpow01_log(xv, p.beta_m1, tail[k], tail[k + 1], l);
                const fl2 r0 = p.want_loss ? vpow01_log(xv, p.beta, tail[k], tail[k + 1], l) : vsplat(0.0f);
                pbm1[k]     = need[k] ? r1[0] : pow01_exact(ax[k], p.beta_m1);
                pbm1[k + 1] = need[k + 1] ? r1[1] : pow01_exact(ax[k + 1], p.beta_m1);
                pb[k]       = need[k] ? r0[0] : pow01_exact(ax[k], p.beta);
                pb[k + 1]   = need[k + 1] ? r0[1] : pow01_exact(ax[k + 1], p.beta);
            }
            else
            {
                pbm1[k]     = pow01_exact(ax[k], p.beta_m1);
                pb[k]       = pow01_exact(ax[k], p.beta);
                pbm1[k + 1] = pow01_exact(ax[k + 1], p.beta_m1);
                pb[k + 1]   = pow01_exact(ax[k + 1], p.beta);
            }
        }
        if constexpr (E % 2 == 1)
        {
            constexpr int k = E - 1;
            if (need[k])
            {
                F2 l {0.0f, 0.0f};
                if (!tail[k])
                    l = sleef_logkf(ax[k]);
                pbm1[k] = pow01_log(ax[k], p.beta_m1, tail[k], l);
                pb[k]   = p.want_loss ? pow01_log(ax[k], p.beta, tail[k], l) : 0.0f;
            }
            else
            {
                pbm1[k] = pow01_exact(ax[k], p.beta_m1);
                pb[k]   = pow01_exact(ax[k], p.beta);
            }
        }
        return;
    }
    uint32_t cnt = 0;
    int pos[E];
#pragma unroll
    for (int k = 0; k < E; ++k)
    {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t) (ballot[k] >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t) ballot[k], 0u));
        pos[k] = need[k] ? (int) (cnt + below) : -1;
        if (need[k])   // |x| >= 0 or NaN: the sign bit marks a tail element
            wl[cnt + below] = tail[k] ? -ax[k] : ax[k];
        cnt += (uint32_t) __popcll(ballot[k]);
    }
    wave_sync();
    float* wl1 = wl + 64 * E;
    // (two entries per lane per pass in packed f32 -- v_pk_fma / v_pk_mul, component-wise the same
    // arithmetic -- measured 2-4 % slower at 2^28 elements, profiles/r04/README.md)
    for (uint32_t j = lane; j < cnt; j += 64)
    {
        const float sv  = wl[j];
        const bool tl   = TAIL && __builtin_signbit(sv);   // a NaN keeps its sign through the negation
        const float v   = __builtin_fabsf(sv);
        if constexpr (EXACT)
        {
            F2 l {0.0f, 0.0f};
            if (!tl)
                l = sleef_logkf(v);
            wl[j] = pow01_log(v, p.beta_m1, tl, l);
            if (p.want_loss)
                wl1[j] = pow01_log(v, p.beta, tl, l);
        }
        else
        {
            const LnSplit l = ln01(v);
            wl[j]          = pow01_fast_l(v, p.beta_m1, l);
            if (p.want_loss)
                wl1[j] = pow01_fast_l(v, p.beta, l);
        }
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < E; ++k)
    {
        if (pos[k] >= 0)
        {
            pbm1[k] = wl[pos[k]];
            pb[k]   = p.want_loss ? wl1[pos[k]] : 0.0f;
        }
        else
        {
            pbm1[k] = pow01_exact(ax[k], p.beta_m1);
            pb[k]   = pow01_exact(ax[k], p.beta);
        }
    }
    wave_sync();   // the slot is reused by the next call
}

// 16-B streaming form: four consecutive elements share a channel (K % 4 == 0 or C == 1);
// one quad per lane, one tile per workgroup (the QDQ kernels' measured-best shape)
__global__ __launch_bounds__(kBlock) void adaround_fwd_vec_kernel(const f4* __restrict__ w, const f4* __restrict__ alpha,
                                                                  f4* __restrict__ wq, uint32_t nq, AdaChannel map,
                                                                  const float* __restrict__ delta,
                                                                  const float* __restrict__ offset, AdaParams p)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nq)
        return;
    const uint32_t c = map.channel(4 * i);
    const float d = delta[c], o = offset[c], rcp = __builtin_amdgcn_rcpf(d);
    f4 wv = __builtin_nontemporal_load(w + i), av = __builtin_nontemporal_load(alpha + i), r;
    r.x = ada_fwd(wv.x, av.x, d, o, p, rcp);
    r.y = ada_fwd(wv.y, av.y, d, o, p, rcp);
    r.z = ada_fwd(wv.z, av.z, d, o, p, rcp);
    r.w = ada_fwd(wv.w, av.w, d, o, p, rcp);
    __builtin_nontemporal_store(r, wq + i);
}

__global__ __launch_bounds__(kBlock) void adaround_fwd_kernel(const float* __restrict__ w,
                                                              const float* __restrict__ alpha, float* __restrict__ wq,
                                                              uint32_t n, AdaChannel map,
                                                              const float* __restrict__ delta,
                                                              const float* __restrict__ offset, AdaParams p)
{
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
    {
        uint32_t c = map.channel(i);
        wq[i]      = ada_fwd(w[i], alpha[i], delta[c], offset[c], p, __builtin_amdgcn_rcpf(delta[c]));
    }
}

__device__ __forceinline__ float block_sum(float v)
{
    __shared__ float s[kBlock / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0)
        s[threadIdx.x >> 6] = v;
    __syncthreads();
    float r = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < kBlock / 64; ++i)
            r += s[i];
    __syncthreads();
    return r;
}

// reg x the sum of the per-workgroup round-loss partials part[0, nparts), added to *round_loss:
// each lane adds its parts in order (kFoldBatch loads in flight), then block_sum's fixed tree --
// one value whatever the workgroups' timing. Called by every thread of one workgroup.
template <bool CONSUME>
__device__ __forceinline__ void round_loss_fold(const float* __restrict__ part, uint32_t nparts, float reg,
                                                float* __restrict__ round_loss)
{
    constexpr int kFoldBatch = 8;
    float t = 0.0f;
    for (uint32_t i0 = threadIdx.x; i0 < nparts; i0 += kBlock * kFoldBatch)
    {
        float v[kFoldBatch];
#pragma unroll
        for (int u = 0; u < kFoldBatch; ++u)
        {
            const uint32_t i = i0 + u * kBlock;
            v[u]             = i < nparts ? (CONSUME ? consume_f32(part + i) : part[i]) : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < kFoldBatch; ++u)
            if (i0 + u * kBlock < nparts)
                t += v[u];
    }
    t = block_sum(t);
    if (threadIdx.x == 0)
        atomicAdd(round_loss, reg * t);
}

// The round loss of one launch: reg x (the per-workgroup sums folded in workgroup order by the
// workgroup that finishes last), one add to *round_loss per launch, so the value does not depend
// on the workgroups' timing (ticket_alloc; `part` holds gridDim.x floats, handed over write-through:
// common.hpp publish_f32). Without a ticket (the capture pool used up: upload.cpp fold_buffers) the
// partials are only stored and round_loss_fold_kernel, launched next, folds them the same way: the
// same value. Called by every thread of every workgroup.
__device__ __forceinline__ void round_loss_add(float loss, float reg, float* __restrict__ round_loss,
                                               float* __restrict__ part, unsigned* __restrict__ ticket)
{
    const float s = block_sum(loss);
    if (!ticket)
    {
        if (threadIdx.x == 0)
            part[blockIdx.x] = s;
        return;
    }
    __shared__ int last;
    if (threadIdx.x == 0)
    {
        publish_f32(part + blockIdx.x, s);
        last = arrive_is_last_grid(ticket);
    }
    __syncthreads();
    if (!last)
        return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the loads below the ticket
    round_loss_fold<true>(part, gridDim.x, reg, round_loss);
    if (threadIdx.x == 0)
        ticket_reset(ticket + kTicketGroups);
}

// the fold of round_loss_add's partials as its own launch (no ticket); reg as the backward read it:
// the argument, reg_beta[0], or (the loop's Adam step) reg_beta[3 (it_next[0] - 1)]
__global__ __launch_bounds__(kBlock) void round_loss_fold_kernel(const float* __restrict__ part, uint32_t nparts,
                                                                 float reg, const float* __restrict__ reg_beta,
                                                                 const int64_t* __restrict__ it_next,
                                                                 float* __restrict__ round_loss)
{
    const float r = reg_beta ? (it_next ? reg_beta[3 * (it_next[0] - 1)] : reg_beta[0]) : reg;
    if (r != 0.0f)
        round_loss_fold<false>(part, nparts, r, round_loss);
}

// backward: grid-stride over tiles of kBlock x U quads (U quads in flight per lane, 3 x 16-B loads
// each; bounded grid: one round-loss atomic per workgroup); the loop bounds are uniform over the
// workgroup (ada_round_pows synchronises it)
// TAIL = false: n % 32 == 0, no element lies in the reference's scalar pow tail (compile-time)
template <int U, bool WL, bool TAIL, bool EXACT>
__global__ __launch_bounds__(kBlock) void adaround_bwd_vec_kernel(const f4* __restrict__ w, const f4* __restrict__ alpha,
                                                                  const f4* __restrict__ g, f4* __restrict__ ga,
                                                                  uint32_t nq, AdaChannel map,
                                                                  const float* __restrict__ delta,
                                                                  const float* __restrict__ offset, AdaParams p,
                                                                  float* __restrict__ round_loss,
                                                                  const float* __restrict__ reg_beta,
                                                                  float* __restrict__ loss_part,
                                                                  unsigned* __restrict__ ticket)
{
    constexpr int E = 4 * U;
    __shared__ float lds[kBlock / 64][2 * 64 * E];
    p.want_loss = WL;   // a constant from here on: the form without the loss value carries none of its work
    if (reg_beta)   // device-resident {reg, beta, beta - 1}: a HIP-graph replay per iteration
    {
        p.reg     = reg_beta[0];
        p.beta    = reg_beta[1];
        p.beta_m1 = reg_beta[2];
    }
    float* wl             = lds[threadIdx.x >> 6];
    float loss            = 0.0f;
    const uint32_t stride = gridDim.x * kBlock * U;
    // the fast pow's tables: their loads first, the LDS copy after the first tile's loads are issued
    PowTabPart<kBlock> tab;
    if constexpr (!EXACT)
        tab = pow_tab_load<kBlock>();
    bool first = true;
    for (uint32_t tile = blockIdx.x * kBlock * U; tile < nq; tile += stride)
    {
        const uint32_t base = tile + threadIdx.x;
        f4 wv[U], av[U], gv[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t i = base + u * kBlock;
            const uint32_t j = i < nq ? i : nq - 1;   // clamped (never stored)
            wv[u] = __builtin_nontemporal_load(w + j);
            av[u] = __builtin_nontemporal_load(alpha + j);
            gv[u] = __builtin_nontemporal_load(g + j);
        }
        if (!EXACT && first)   // uniform over the workgroup
        {
            pow_tab_store<kBlock>(tab);
            __syncthreads();
            first = false;
        }
        float r[E], sg[E], x[E], ax[E];
        bool in_h[E], tail[E], valid[E];
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t i = base + u * kBlock;
            const uint32_t c = map.channel(4 * (i < nq ? i : nq - 1));
            const float d = delta[c], o = offset[c], rcp = __builtin_amdgcn_rcpf(d);
            const float wu[4] = {wv[u].x, wv[u].y, wv[u].z, wv[u].w}, au[4] = {av[u].x, av[u].y, av[u].z, av[u].w},
                        gu[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
            {
                const int k = 4 * u + e;
                r[k]     = ada_bwd_base(wu[e], au[e], gu[e], d, o, p, rcp, sg[k], x[k], in_h[k]);
                ax[k]    = fabsf(x[k]);
                valid[k] = i < nq;
                in_h[k]  = in_h[k] && valid[k];
                tail[k]  = 4 * i + e >= p.vec_end;
            }
        }
        if (p.reg != 0.0f)   // uniform: a kernel argument or the device-resident value
        {
            float pbm1[E], pb[E];
            ada_round_pows<E, TAIL, EXACT>(ax, tail, p.want_loss ? valid : in_h, p, wl, pbm1, pb);
#pragma unroll
            for (int k = 0; k < E; ++k)
                if (p.want_loss && valid[k])
                    loss += 1.0f - pb[k];
            if (p.reg > 0.0f && p.beta > 0.0f && p.beta_m1 > 0.0f)   // uniform: every schedule's case
            {
#pragma unroll
                for (int k = 0; k < E; ++k)
                    r[k] = ada_bwd_round<true>(r[k], sg[k], x[k], in_h[k], pbm1[k], p);
            }
            else
            {
#pragma unroll
                for (int k = 0; k < E; ++k)
                    r[k] = ada_bwd_round(r[k], sg[k], x[k], in_h[k], pbm1[k], p);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
        {
            const uint32_t i = base + u * kBlock;
            if (i < nq)
                __builtin_nontemporal_store(f4 {r[4 * u], r[4 * u + 1], r[4 * u + 2], r[4 * u + 3]}, ga + i);
        }
    }
    if (p.reg != 0.0f && round_loss)
        round_loss_add(loss, p.reg, round_loss, loss_part, ticket);
}

template <bool EXACT>
__global__ __launch_bounds__(kBlock) void adaround_bwd_kernel(const float* __restrict__ w,
                                                              const float* __restrict__ alpha,
                                                              const float* __restrict__ g, float* __restrict__ ga,
                                                              uint32_t n, AdaChannel map,
                                                              const float* __restrict__ delta,
                                                              const float* __restrict__ offset, AdaParams p,
                                                              float* __restrict__ round_loss,
                                                              const float* __restrict__ reg_beta,
                                                              float* __restrict__ loss_part, unsigned* __restrict__ ticket)
{
    if (reg_beta)
    {
        p.reg     = reg_beta[0];
        p.beta    = reg_beta[1];
        p.beta_m1 = reg_beta[2];
    }
    if constexpr (!EXACT)
    {
        pow_tab_fill<kBlock>();
        __syncthreads();
    }
    float loss = 0.0f;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
    {
        uint32_t c = map.channel(i);
        ga[i]      = ada_bwd<EXACT>(w[i], alpha[i], g[i], delta[c], offset[c], p, __builtin_amdgcn_rcpf(delta[c]), loss, i);
    }
    if (p.reg != 0.0f && round_loss)
        round_loss_add(loss, p.reg, round_loss, loss_part, ticket);
}

// the round loss's per-workgroup partials and completion ticket for one launch (round_loss_add);
// none when no loss is requested. Without a ticket (the capture pool used up), partials from the
// scratch allocator (a graph memory node inside a capture) and a fold launch after the kernel
// (finish()): the same value either way. The partials are released after the launch that uses them.
struct LossFold
{
    float* part      = nullptr;
    unsigned* ticket = nullptr;
    FoldBuffers fb;
    hipStream_t s;
    unsigned grid = 0;
    bool scratch  = false;
    LossFold(const float* round_loss, unsigned g, hipStream_t st) : s(st), grid(g)
    {
        if (!round_loss)
            return;
        fb     = fold_buffers(st, kTicketGroups + 1, grid);
        ticket = fb.ticket;
        part   = fb.part;
        if (!ticket)
        {
            part    = static_cast<float*>(scratch_alloc(sizeof(float) * grid, st));
            scratch = true;
        }
    }
    // after the backward's launch: the fold of its partials when they had no ticket
    void finish(float reg, const float* reg_beta, const int64_t* it_next, float* round_loss)
    {
        if (!scratch)
            return;
        round_loss_fold_kernel<<<1, kBlock, 0, s>>>(part, grid, reg, reg_beta, it_next, round_loss);
        AIMET_LAUNCH_CHECK();
    }
    ~LossFold()
    {
        try
        {
            if (scratch)
                scratch_free(part, s);
            fold_buffers_release(fb, s);
        }
        catch (...)   // a failing event record: the block is leaked, never handed out again
        {
        }
    }
    LossFold(const LossFold&)            = delete;
    LossFold& operator=(const LossFold&) = delete;
};

bool aligned16(const void* p)
{
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0;
}

// the rounding loss's pow for launches from now on: the fast pow (0, default) or the bit-exact
// emulation of torch's (1); aimet_adaround_set_exact_pow
std::atomic<int>& exact_pow_flag()
{
    static std::atomic<int> f {0};
    return f;
}
bool exact_pow()
{
    return exact_pow_flag().load(std::memory_order_relaxed) != 0;
}

// ---- one optimizer step fused into the backward (single-process HIP-graph loop) -----------------
// torch.optim.Adam(fused=True) per element, as ATen's adam_math (native/hip/fused_adam_utils.cuh)
// computes it for a float parameter without weight decay / amsgrad / maximize: the moments in
// double (double betas times float values), rounded to float; step size and denominator as there.
struct AdamArgs
{
    double lr, beta1, beta2, eps;
};

__device__ __forceinline__ float adam_elem(float param, float grad, float& exp_avg, float& exp_avg_sq,
                                           const AdamArgs& a, float bias_correction1, float bias_correction2_sqrt)
{
    exp_avg               = a.beta1 * exp_avg + (1 - a.beta1) * grad;
    exp_avg_sq            = a.beta2 * exp_avg_sq + (1 - a.beta2) * grad * grad;
    const float step_size = a.lr / bias_correction1;
    const float denom     = (std::sqrt(exp_avg_sq) / bias_correction2_sqrt) + a.eps;
    param -= step_size * exp_avg / denom;
    return param;
}

// ATen: 1 - pow_(beta, float step) in double, handed to adam_math as float (bias_correction2 as
// its square root); one definition for the in-kernel path and the per-step table, so both give
// the same bits
__device__ __forceinline__ void adam_bias_corrections(double beta1, double beta2, int64_t step, float& bc1,
                                                      float& bc2s)
{
    const float step_f = (float) step;
    bc1                = (float) (1 - pow(beta1, (double) step_f));
    bc2s               = (float) sqrt(1 - pow(beta2, (double) step_f));
}

// bias_corr[2 (step - 1) ..] = {bc1, bc2s} for step = 1 .. steps
__global__ __launch_bounds__(kBlock) void adam_bias_corr_kernel(double beta1, double beta2, int64_t steps,
                                                                float* __restrict__ bias_corr)
{
    const int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (i < steps)
        adam_bias_corrections(beta1, beta2, i + 1, bias_corr[2 * i], bias_corr[2 * i + 1]);
}

// dL/dalpha (ada_bwd, with this iteration's {reg, beta, beta - 1} from reg_beta_all[it]) and the
// Adam update of alpha in place; `step` = it_next[0] (= it + 1, written by the gather kernel of the
// same iteration), workgroup 0 publishes it to it_cur for the next iteration's gather.
template <bool VEC, bool WL, bool TAIL, bool EXACT>
__global__ __launch_bounds__(kBlock) void adaround_bwd_adam_kernel(const float* __restrict__ w,
                                                                   float* __restrict__ alpha,
                                                                   const float* __restrict__ g,
                                                                   float* __restrict__ exp_avg,
                                                                   float* __restrict__ exp_avg_sq, uint32_t n,
                                                                   AdaChannel map, const float* __restrict__ delta,
                                                                   const float* __restrict__ offset, AdaParams p,
                                                                   const float* __restrict__ reg_beta_all,
                                                                   const int64_t* __restrict__ it_next,
                                                                   int64_t* __restrict__ it_cur, AdamArgs adam,
                                                                   float* __restrict__ round_loss,
                                                                   float* __restrict__ wq_next,
                                                                   float* __restrict__ loss_part,
                                                                   unsigned* __restrict__ ticket, uint32_t nparts,
                                                                   const float* __restrict__ bias_corr,
                                                                   uint32_t part_kk)
{
    p.want_loss = WL;   // constant: see adaround_bwd_vec_kernel
    // the fast pow's tables: loaded first, copied into LDS once the step's operands are in flight
    PowTabPart<kBlock> tab;
    if constexpr (!EXACT)
        tab = pow_tab_load<kBlock>();
    // the one-element-per-lane form's first element: its operands are loaded before the step's
    // table entries, which they do not depend on, so the two round trips overlap (a small layer's
    // step is a chain of latencies: the counter, the table entries, the operands, the arithmetic)
    const uint32_t i0 = blockIdx.x * kBlock + threadIdx.x;
    // slice s of element i's gradient: [nparts][n] (slice-major), or [n / part_kk][nparts][part_kk]
    // (the depthwise step's per-channel slices; the first slice added to +0 as dw_wgrad_fold does,
    // so the sum is that fold's bit for bit)
    auto gpart = [&](uint32_t i, uint32_t sl) -> float {
        if (part_kk)
        {
            const uint32_t ch = i / part_kk, k = i - ch * part_kk;
            const float v     = g[((size_t) ch * nparts + sl) * part_kk + k];
            return sl == 0 ? 0.0f + v : v;
        }
        return g[(size_t) sl * n + i];
    };
    float f_w = 0.0f, f_a = 0.0f, f_g = 0.0f, f_m = 0.0f, f_v = 0.0f, f_d = 1.0f, f_o = 0.0f;
    if (!VEC && i0 < n)
    {
        const uint32_t c = map.channel(i0);
        f_d              = delta[c];
        f_o              = offset[c];
        f_w              = w[i0];
        f_a              = alpha[i0];
        f_g              = gpart(i0, 0);
        f_m              = exp_avg[i0];
        f_v              = exp_avg_sq[i0];
    }
    const int64_t step = it_next[0];
    if (blockIdx.x == 0 && threadIdx.x == 0)
        it_cur[0] = step;
    const float* rb = reg_beta_all + 3 * (step - 1);
    p.reg           = rb[0];
    p.beta          = rb[1];
    p.beta_m1       = rb[2];
    // ATen's bias corrections: from the per-step table when given (two loads instead of ~540
    // dependent f64 instructions ahead of every wave's first element), else computed here
    float bc1, bc2s;
    if (bias_corr)
    {
        bc1  = bias_corr[2 * (step - 1)];
        bc2s = bias_corr[2 * (step - 1) + 1];
    }
    else
        adam_bias_corrections(adam.beta1, adam.beta2, step, bc1, bc2s);
    if constexpr (!EXACT)
    {
        pow_tab_store<kBlock>(tab);
        __syncthreads();
    }
    float loss         = 0.0f;
    if (VEC)
    {
        // one quad per lane; the rounding-loss pows wave-compacted (ada_round_pows), so the loop
        // bounds are uniform over the workgroup
        __shared__ float lds[kBlock / 64][2 * 64 * 4];
        float* wl         = lds[threadIdx.x >> 6];
        const uint32_t nq = n / 4;
        for (uint32_t i0 = blockIdx.x * kBlock; i0 < nq; i0 += gridDim.x * kBlock)
        {
            const uint32_t i  = i0 + threadIdx.x;
            const bool valid  = i < nq;
            const uint32_t ic = valid ? i : nq - 1;   // clamped (never stored)
            const uint32_t c  = map.channel(4 * ic);
            const float d = delta[c], o = offset[c], rcp = __builtin_amdgcn_rcpf(d);
            f4 wv       = __builtin_nontemporal_load(reinterpret_cast<const f4*>(w) + ic);
            f4 gv       = __builtin_nontemporal_load(reinterpret_cast<const f4*>(g) + ic);
            // the gradient's slices, added in slice order; up to 8 loads in flight at a time
            for (uint32_t s = 1; s < nparts; s += 8)
            {
                f4 t[8];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    t[u] = __builtin_nontemporal_load(
                        reinterpret_cast<const f4*>(g + (size_t) (s + u < nparts ? s + u : s) * n) + ic);
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (s + u < nparts)
                        gv += t[u];
            }
            f4 av       = reinterpret_cast<const f4*>(alpha)[ic];
            float a[4] = {av.x, av.y, av.z, av.w}, ww[4] = {wv.x, wv.y, wv.z, wv.w}, gg[4] = {gv.x, gv.y, gv.z, gv.w};
            float r[4], sg[4], x[4], ax[4];
            bool in_h[4], tail[4], use[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
            {
                r[k]    = ada_bwd_base(ww[k], a[k], gg[k], d, o, p, rcp, sg[k], x[k], in_h[k]);
                ax[k]   = fabsf(x[k]);
                in_h[k] = in_h[k] && valid;
                tail[k] = 4 * ic + k >= p.vec_end;
                use[k]  = p.want_loss ? valid : in_h[k];
            }
            if (p.reg != 0.0f)   // uniform: this iteration's device-resident value
            {
                float pbm1[4], pb[4];
                ada_round_pows<4, TAIL, EXACT>(ax, tail, use, p, wl, pbm1, pb);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                {
                    if (p.want_loss && valid)
                        loss += 1.0f - pb[k];
                    r[k] = ada_bwd_round(r[k], sg[k], x[k], in_h[k], pbm1[k], p);
                }
            }
            if (!valid)
                continue;
            f4 mv      = reinterpret_cast<const f4*>(exp_avg)[i];
            f4 vv      = reinterpret_cast<const f4*>(exp_avg_sq)[i];
            float m[4] = {mv.x, mv.y, mv.z, mv.w}, v[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                a[k] = adam_elem(a[k], r[k], m[k], v[k], adam, bc1, bc2s);
            reinterpret_cast<f4*>(alpha)[i]      = f4 {a[0], a[1], a[2], a[3]};
            reinterpret_cast<f4*>(exp_avg)[i]    = f4 {m[0], m[1], m[2], m[3]};
            reinterpret_cast<f4*>(exp_avg_sq)[i] = f4 {v[0], v[1], v[2], v[3]};
            if (wq_next)   // the next iteration's soft-quantized weight from the updated alpha
                __builtin_nontemporal_store(f4 {ada_fwd(ww[0], a[0], d, o, p, rcp), ada_fwd(ww[1], a[1], d, o, p, rcp),
                                                ada_fwd(ww[2], a[2], d, o, p, rcp), ada_fwd(ww[3], a[3], d, o, p, rcp)},
                                            reinterpret_cast<f4*>(wq_next) + i);
        }
    }
    else
    {
        for (uint32_t i = i0; i < n; i += gridDim.x * kBlock)
        {
            float d = f_d, o = f_o, wi = f_w, ai = f_a, gi = f_g, mi = f_m, vi = f_v;
            if (i != i0)
            {
                const uint32_t c = map.channel(i);
                d                = delta[c];
                o                = offset[c];
                wi               = w[i];
                ai               = alpha[i];
                gi               = gpart(i, 0);
                mi               = exp_avg[i];
                vi               = exp_avg_sq[i];
            }
            const float rcp = __builtin_amdgcn_rcpf(d);
            for (uint32_t s = 1; s < nparts; s += 16)   // slice order; up to 16 loads in flight
            {
                float t[16];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    t[u] = gpart(i, s + u < nparts ? s + u : s);
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (s + u < nparts)
                        gi += t[u];
            }
            const float ga  = ada_bwd<EXACT>(wi, ai, gi, d, o, p, rcp, loss, i);
            const float an  = adam_elem(ai, ga, mi, vi, adam, bc1, bc2s);
            alpha[i]        = an;
            exp_avg[i]      = mi;
            exp_avg_sq[i]   = vi;
            if (wq_next)
                wq_next[i] = ada_fwd(wi, an, d, o, p, rcp);
        }
    }
    if (p.reg != 0.0f && round_loss)
        round_loss_add(loss, p.reg, round_loss, loss_part, ticket);
}

// this iteration's batch: rows idx_all[it][b] of the cached inputs / outputs -> dst_in[b] /
// dst_out[b] (blockIdx.y = 2 b + which); it = it_cur[0]; workgroup (0, 0) sets it_next = it + 1
__global__ __launch_bounds__(kBlock) void adaround_gather_kernel(const float* __restrict__ src_in,
                                                                 const float* __restrict__ src_out,
                                                                 float* __restrict__ dst_in, float* __restrict__ dst_out,
                                                                 const int64_t* __restrict__ idx_all,
                                                                 const int64_t* __restrict__ it_cur,
                                                                 int64_t* __restrict__ it_next, int nb, int64_t row_in,
                                                                 int64_t row_out, int vec)
{
    const int64_t it = it_cur[0];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
        it_next[0] = it + 1;
    const int b          = blockIdx.y >> 1;
    const bool out       = blockIdx.y & 1;
    if (out ? !dst_out : !dst_in)
        return;   // read in place (recon_grad_idx_kernel, the depthwise kernels' row map)
    const int64_t row    = out ? row_out : row_in;
    const int64_t r      = idx_all[it * nb + b];
    const float* src     = (out ? src_out : src_in) + r * row;
    float* dst           = (out ? dst_out : dst_in) + (int64_t) b * row;
    const int64_t stride = (int64_t) gridDim.x * kBlock;
    if (vec)
    {
        const f4* s4 = reinterpret_cast<const f4*>(src);
        f4* d4       = reinterpret_cast<f4*>(dst);
        for (int64_t q = (int64_t) blockIdx.x * kBlock + threadIdx.x; q < row / 4; q += stride)
            d4[q] = __builtin_nontemporal_load(s4 + q);
    }
    else
        for (int64_t q = (int64_t) blockIdx.x * kBlock + threadIdx.x; q < row; q += stride)
            dst[q] = src[q];
}

// ---- reconstruction-loss gradient (adaround_loss.py:70-80; recon_g in recon.hpp) --------------
// one elementwise pass (12 B/elem) for the ~12 torch kernels of act / sub / norm / pow / mean and
// their backward.
__global__ __launch_bounds__(kBlock) void recon_grad_vec_kernel(const f4* __restrict__ q, const f4* __restrict__ t,
                                                                f4* __restrict__ g, int64_t nq, float scale, int act)
{
    const int64_t i = (int64_t) blockIdx.x * kBlock + threadIdx.x;
    if (i >= nq)
        return;
    const f4 a = __builtin_nontemporal_load(q + i), b = __builtin_nontemporal_load(t + i);
    f4 r;
    r.x = recon_g(a.x, b.x, scale, act);
    r.y = recon_g(a.y, b.y, scale, act);
    r.z = recon_g(a.z, b.z, scale, act);
    r.w = recon_g(a.w, b.w, scale, act);
    __builtin_nontemporal_store(r, g + i);
}

__global__ __launch_bounds__(kBlock) void recon_grad_kernel(const float* __restrict__ q, const float* __restrict__ t,
                                                            float* __restrict__ g, int64_t begin, int64_t n,
                                                            float scale, int act)
{
    for (int64_t i = begin + (int64_t) blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t) gridDim.x * kBlock)
        g[i] = recon_g(q[i], t[i], scale, act);
}

// recon_grad with the fp target read in place from the cached outputs (row idx_all[it][b] for
// sample b, it = it_cur[0]) and, optionally, the layer bias added to q first (q = the bias-free
// GEMM output; channel = (i / hw) % C of the [nb][C][hw] batch): no gathered copy of the target,
// no separate bias pass
struct ReconIdx
{
    const float* out_data;
    const int64_t* idx_all;
    const int64_t* it_cur;
    const float* bias;   // nullable
    int64_t nb, row, hw, C;
    FastDiv div_row, div_hw, div_c;
};

__device__ __forceinline__ float recon_bias(const ReconIdx& r, uint32_t e_in_row)
{
    if (!r.bias)
        return 0.0f;
    const uint32_t ch = r.div_hw.div(e_in_row);
    return r.bias[ch - r.div_c.div(ch) * (uint32_t) r.C];
}

// Channel-major batches of a 1x1 layer's GEMM form: x_cm[ci][b][hw] = src_in[idx[it][b]][ci][hw]
// (one GEMM over all positions then gives q_cm[co][b][hw] and the weight gradient
// g_cm[co][(b, hw)] x_cm[ci][(b, hw)]^T, no per-sample GEMMs and no batch sum). Flat over the
// destination, PER consecutive elements per lane (4 when hw % 4 == 0: one 16-B load and store,
// the quad inside one plane); a workgroup per (ci, b) plane of 49..196 floats ran at 11 us for
// 1.6 MB. Workgroup 0 sets it_next = it + 1.
template <int PER>
__global__ __launch_bounds__(kBlock) void adaround_gather_cm_kernel(const float* __restrict__ src_in,
                                                                    float* __restrict__ dst,
                                                                    const int64_t* __restrict__ idx_all,
                                                                    const int64_t* __restrict__ it_cur,
                                                                    int64_t* __restrict__ it_next, uint32_t nb,
                                                                    uint32_t Cin, uint32_t hw, uint32_t n,
                                                                    FastDiv div_hw, FastDiv div_nb)
{
    const int64_t it = it_cur[0];
    if (blockIdx.x == 0 && threadIdx.x == 0)
        it_next[0] = it + 1;
    const uint32_t i = (blockIdx.x * kBlock + threadIdx.x) * PER;
    if (i >= n)
        return;
    const uint32_t row = div_hw.div(i), t = i - row * hw;   // row = ci * nb + b
    const uint32_t ci = div_nb.div(row), b = row - ci * nb;
    const float* src  = src_in + ((size_t) idx_all[it * nb + b] * Cin + ci) * hw + t;
    if constexpr (PER == 4)
        *reinterpret_cast<f4*>(dst + i) = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src));
    else
        dst[i] = __builtin_nontemporal_load(src);
}

// recon_grad_idx_kernel for channel-major q / g ([C][nb][hw]): element i = (co nb + b) hw + t reads
// the target out_data[idx[it][b]][co][t]; bias added first as there. PER = 4 when hw % 4 == 0.
template <int PER>
__global__ __launch_bounds__(kBlock) void recon_grad_idx_cm_kernel(const float* __restrict__ q, float* __restrict__ g,
                                                                   ReconIdx r, float scale, int act)
{
    const int64_t it   = r.it_cur[0];
    const uint32_t n   = (uint32_t) (r.C * r.nb * r.hw);
    const uint32_t i   = (blockIdx.x * kBlock + threadIdx.x) * PER;
    if (i >= n)
        return;
    const uint32_t row = r.div_hw.div(i);   // co * nb + b
    const uint32_t t   = i - row * (uint32_t) r.hw;
    const uint32_t co  = r.div_c.div(row);   // div_c holds nb here
    const uint32_t b   = row - co * (uint32_t) r.nb;
    const float* tp    = r.out_data + ((size_t) r.idx_all[it * r.nb + b] * r.C + co) * r.hw + t;
    const float bs     = r.bias ? r.bias[co] : 0.0f;
    if constexpr (PER == 4)
    {
        const f4 a = __builtin_nontemporal_load(reinterpret_cast<const f4*>(q + i));
        const f4 c = __builtin_nontemporal_load(reinterpret_cast<const f4*>(tp));
        *reinterpret_cast<f4*>(g + i) = f4 {recon_g(a.x + bs, c.x, scale, act), recon_g(a.y + bs, c.y, scale, act),
                                            recon_g(a.z + bs, c.z, scale, act), recon_g(a.w + bs, c.w, scale, act)};
    }
    else
        g[i] = recon_g(q[i] + bs, *tp, scale, act);
}

template <bool VEC>
__global__ __launch_bounds__(kBlock) void recon_grad_idx_kernel(const float* __restrict__ q, float* __restrict__ g,
                                                                ReconIdx r, float scale, int act)
{
    const int64_t it    = r.it_cur[0];
    const uint32_t per  = VEC ? 4 : 1;
    const uint32_t n    = (uint32_t) (r.nb * r.row);
    const uint32_t i    = (blockIdx.x * kBlock + threadIdx.x) * per;
    if (i >= n)
        return;
    const uint32_t b    = r.div_row.div(i);
    const uint32_t e    = i - b * (uint32_t) r.row;
    const float* t      = r.out_data + r.idx_all[it * r.nb + b] * r.row + e;
    if (VEC)
    {
        const f4 a = __builtin_nontemporal_load(reinterpret_cast<const f4*>(q + i));
        const f4 c = __builtin_nontemporal_load(reinterpret_cast<const f4*>(t));
        const float bs = recon_bias(r, e);   // hw % 4 == 0: the quad shares its channel
        f4 o;
        o.x = recon_g(a.x + bs, c.x, scale, act);
        o.y = recon_g(a.y + bs, c.y, scale, act);
        o.z = recon_g(a.z + bs, c.z, scale, act);
        o.w = recon_g(a.w + bs, c.w, scale, act);
        __builtin_nontemporal_store(o, reinterpret_cast<f4*>(g + i));
    }
    else
        g[i] = recon_g(q[i] + recon_bias(r, e), t[0], scale, act);
}


}   // namespace
}   // namespace aimet_amd

using namespace aimet_amd;

extern "C" {

int aimet_adaround_forward(const float* w, const float* alpha, float* wq, int64_t outer, int64_t C, int64_t K,
                           const float* delta, const float* offset, int32_t bw, int soft, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        int64_t n = outer * C * K;
        if (n == 0)
            return;
        AIMET_REQUIRE(n < (int64_t(1) << 31), "AdaRound weight too large (>= 2^31 elements)");
        require_device_ptr(w, "weight");
        require_device_ptr(alpha, "alpha");
        require_device_ptr(wq, "output");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        AdaChannel map {FastDiv((uint32_t) (K > 0 ? K : 1)), FastDiv((uint32_t) C), (uint32_t) C};
        AdaParams p {(float) ((1ull << bw) - 1), 0.0f, 0.0f, 0.0f, soft, (uint32_t) (n - n % 32), 0};
        if ((C == 1 || K % 4 == 0) && n % 4 == 0 && aligned16(w) && aligned16(alpha) && aligned16(wq))
        {
            uint32_t nq = (uint32_t) (n / 4);
            adaround_fwd_vec_kernel<<<ceil_div(nq, kBlock), kBlock, 0, as_stream(stream)>>>(
                reinterpret_cast<const f4*>(w), reinterpret_cast<const f4*>(alpha), reinterpret_cast<f4*>(wq), nq,
                map, delta, offset, p);
        }
        else
            adaround_fwd_kernel<<<stream_blocks(n, kBlock), kBlock, 0, as_stream(stream)>>>(
                w, alpha, wq, (uint32_t) n, map, delta, offset, p);
        AIMET_LAUNCH_CHECK();
    });
}

}   // extern "C"

namespace
{

int adaround_backward(const float* w, const float* alpha, const float* g, float* ga, int64_t outer, int64_t C,
                      int64_t K, const float* delta, const float* offset, int32_t bw, double reg, double beta,
                      const float* reg_beta, float* round_loss, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        int64_t n = outer * C * K;
        if (n == 0)
            return;
        AIMET_REQUIRE(n < (int64_t(1) << 31), "AdaRound weight too large (>= 2^31 elements)");
        require_device_ptr(w, "weight");
        require_device_ptr(alpha, "alpha");
        require_device_ptr(g, "grad");
        require_device_ptr(ga, "grad_alpha");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        AdaChannel map {FastDiv((uint32_t) (K > 0 ? K : 1)), FastDiv((uint32_t) C), (uint32_t) C};
        if ((float) reg == 0.0f && !reg_beta)   // the kernels add no loss term at reg 0: no partials to fold
            round_loss = nullptr;
        AdaParams p {(float) ((1ull << bw) - 1), (float) reg, (float) beta, (float) (beta - 1.0), 1,
                     (uint32_t) (n - n % 32), round_loss != nullptr};
        hipStream_t st = as_stream(stream);
        if ((C == 1 || K % 4 == 0) && n % 4 == 0 && aligned16(w) && aligned16(alpha) && aligned16(g) &&
            aligned16(ga))
        {
            uint32_t nq = (uint32_t) (n / 4);
            // quads in flight per lane (round 4 with the exact pow: 1 measured best, 2 equal within
            // noise, 4 slower: profiles/r04/ada_bwd_tune_tail_flag.jsonl); a study build may set it
            constexpr int U   = AIMET_ADA_BWD_U;
            int64_t blocks    = ceil_div(nq, kBlock * U);
            // one tile per workgroup unless round-loss partials are folded (one per workgroup): a
            // grid-stride loop over 8192 workgroups holds the 3-read + 1-write stream to 0.60 of
            // 8 TB/s, a full grid reaches 0.78-0.82 (tools/studies/stream_mix.hip); without the
            // pow (reg 0) the kernel follows, 0.58 -> 0.79-0.82 (profiles/r05/ada_bwd_grid.jsonl)
            const int64_t cap = round_loss ? kAdaBwdGrid : blocks;
            const unsigned gx = (unsigned) (blocks < cap ? blocks : cap);
            LossFold lf(round_loss, gx, st);
            auto launch = [&](auto kernel) {
                kernel<<<gx, kBlock, 0, st>>>(
                    reinterpret_cast<const f4*>(w), reinterpret_cast<const f4*>(alpha), reinterpret_cast<const f4*>(g),
                    reinterpret_cast<f4*>(ga), nq, map, delta, offset, p, round_loss, reg_beta, lf.part, lf.ticket);
            };
            // the scalar pow tail exists only for the exact pow (the fast pow takes every element alike)
            const bool wl = p.want_loss != 0, ex = exact_pow(), tl = ex && n % 32 != 0;
            // (a form compiled for 8 waves per SIMD spilled and measured slower:
            // profiles/r04/ada_bwd_tune_occ8.jsonl)
            auto go = [&](auto u) {
                constexpr int UU = decltype(u)::value;
                if (!ex)
                    wl ? launch(adaround_bwd_vec_kernel<UU, true, false, false>)
                       : launch(adaround_bwd_vec_kernel<UU, false, false, false>);
                else if (tl)
                    wl ? launch(adaround_bwd_vec_kernel<UU, true, true, true>)
                       : launch(adaround_bwd_vec_kernel<UU, false, true, true>);
                else
                    wl ? launch(adaround_bwd_vec_kernel<UU, true, false, true>)
                       : launch(adaround_bwd_vec_kernel<UU, false, false, true>);
            };
            go(std::integral_constant<int, U> {});
            AIMET_LAUNCH_CHECK();
            lf.finish(p.reg, reg_beta, nullptr, round_loss);
        }
        else
        {
            const unsigned gx = stream_blocks(n, kBlock);
            LossFold lf(round_loss, gx, st);
            auto launch = [&](auto kernel) {
                kernel<<<gx, kBlock, 0, st>>>(w, alpha, g, ga, (uint32_t) n, map, delta, offset, p, round_loss, reg_beta,
                                              lf.part, lf.ticket);
            };
            exact_pow() ? launch(adaround_bwd_kernel<true>) : launch(adaround_bwd_kernel<false>);
            AIMET_LAUNCH_CHECK();
            lf.finish(p.reg, reg_beta, nullptr, round_loss);
        }
    });
}

}   // namespace

extern "C" {

int aimet_adaround_backward(const float* w, const float* alpha, const float* g, float* ga, int64_t outer, int64_t C,
                            int64_t K, const float* delta, const float* offset, int32_t bw, double reg, double beta,
                            float* round_loss, void* stream)
{
    return adaround_backward(w, alpha, g, ga, outer, C, K, delta, offset, bw, reg, beta, nullptr, round_loss, stream);
}

int aimet_adaround_recon_grad(const float* q, const float* t, float* g, int64_t n, int64_t reduced, int act,
                              void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(n >= 0 && reduced > 0, "invalid shape");
        AIMET_REQUIRE(act >= 0 && act <= 2, "act must be 0 (none), 1 (ReLU) or 2 (ReLU6)");
        if (n == 0)
            return;
        require_device_ptr(q, "quant_out");
        require_device_ptr(t, "orig_out");
        require_device_ptr(g, "grad");
        AIMET_REQUIRE(n % reduced == 0, "element count is not a multiple of the reduced dimension");
        // torch: mean over n / reduced values of the dim-1 squared norm; d/dq = 2 (a - b) / count
        const float scale = (float) (2.0 / (double) (n / reduced));
        hipStream_t s     = as_stream(stream);
        int64_t done      = 0;
        if (aligned16(q) && aligned16(t) && aligned16(g))
        {
            const int64_t nq = n / 4;
            if (nq)
            {
                AIMET_REQUIRE(ceil_div(nq, kBlock) < (int64_t(1) << 31), "tensor too large");
                recon_grad_vec_kernel<<<(unsigned) ceil_div(nq, kBlock), kBlock, 0, s>>>(
                    reinterpret_cast<const f4*>(q), reinterpret_cast<const f4*>(t), reinterpret_cast<f4*>(g), nq,
                    scale, act);
                AIMET_LAUNCH_CHECK();
            }
            done = nq * 4;
        }
        if (done < n)
        {
            recon_grad_kernel<<<stream_blocks(n - done, kBlock), kBlock, 0, s>>>(q, t, g, done, n, scale, act);
            AIMET_LAUNCH_CHECK();
        }
    });
}

int aimet_adaround_backward_dev(const float* w, const float* alpha, const float* g, float* ga, int64_t outer,
                                int64_t C, int64_t K, const float* delta, const float* offset, int32_t bw,
                                const float* reg_beta_dev, float* round_loss, void* stream)
{
    const int rc = guarded([&] {
        AIMET_REQUIRE(reg_beta_dev != nullptr, "reg_beta_dev is null");
        require_device_ptr(reg_beta_dev, "reg_beta");
    });
    if (rc != AIMET_OK)
        return rc;
    return adaround_backward(w, alpha, g, ga, outer, C, K, delta, offset, bw, 0.0, 0.0, reg_beta_dev, round_loss,
                             stream);
}

}   // extern "C"

extern "C" {

int aimet_adaround_gather(const float* src_in, const float* src_out, float* dst_in, float* dst_out,
                          const int64_t* idx_all, const int64_t* it_cur, int64_t* it_next, int64_t nb, int64_t row_in,
                          int64_t row_out, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(nb > 0 && nb <= 32768 && row_in > 0 && row_out > 0, "invalid batch / row sizes");
        require_device_ptr(src_in, "src_in");
        require_device_ptr(src_out, "src_out");
        if (dst_in)    // null: the inputs are read in place (only the iteration counter moves)
            require_device_ptr(dst_in, "dst_in");
        if (dst_out)   // null: the targets are read in place
            require_device_ptr(dst_out, "dst_out");
        require_device_ptr(idx_all, "idx_all");
        require_device_ptr(it_cur, "it_cur");
        require_device_ptr(it_next, "it_next");
        const bool vec = row_in % 4 == 0 && row_out % 4 == 0 && aligned16(src_in) && aligned16(src_out) &&
                         aligned16(dst_in) && aligned16(dst_out);   // aligned16(nullptr) holds
        const int64_t rin  = dst_in ? row_in : 0, rout = dst_out ? row_out : 0;
        const int64_t work = (rin > rout ? rin : rout) / (vec ? 4 : 1);
        int64_t bx         = ceil_div(work, kBlock * 4);   // >= 4 items per lane
        bx                 = bx < 1 ? 1 : (bx > 256 ? 256 : bx);
        dim3 grid((unsigned) bx, (unsigned) (2 * nb));
        adaround_gather_kernel<<<grid, kBlock, 0, as_stream(stream)>>>(src_in, src_out, dst_in, dst_out, idx_all,
                                                                        it_cur, it_next, (int) nb, row_in, row_out,
                                                                        vec ? 1 : 0);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_adaround_recon_grad_indexed(const float* q, const float* out_data, const int64_t* idx_all,
                                      const int64_t* it_cur, float* g, int64_t nb, int64_t C, int64_t hw,
                                      const float* bias, int act, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(nb > 0 && C > 0 && hw > 0, "invalid shape");
        AIMET_REQUIRE(act >= 0 && act <= 2, "act must be 0 (none), 1 (ReLU) or 2 (ReLU6)");
        const int64_t row = C * hw, n = nb * row;
        AIMET_REQUIRE(n < (int64_t(1) << 31), "batch too large (>= 2^31 elements)");
        require_device_ptr(q, "quant_out");
        require_device_ptr(out_data, "out_data");
        require_device_ptr(idx_all, "idx_all");
        require_device_ptr(it_cur, "it_cur");
        require_device_ptr(g, "grad");
        if (bias)
            require_device_ptr(bias, "bias");
        // torch: mean over n / C values of the dim-1 squared norm; d/dq = 2 (a - b) / count
        const float scale = (float) (2.0 / (double) (n / C));
        ReconIdx r {out_data, idx_all, it_cur, bias, nb, row, hw, C,
                    FastDiv((uint32_t) row), FastDiv((uint32_t) hw), FastDiv((uint32_t) C)};
        const bool vec = row % 4 == 0 && hw % 4 == 0 && aligned16(q) && aligned16(out_data) && aligned16(g);
        hipStream_t s  = as_stream(stream);
        if (vec)
            recon_grad_idx_kernel<true><<<(unsigned) ceil_div(n / 4, kBlock), kBlock, 0, s>>>(q, g, r, scale, act);
        else
            recon_grad_idx_kernel<false><<<(unsigned) ceil_div(n, kBlock), kBlock, 0, s>>>(q, g, r, scale, act);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_adaround_gather_cm(const float* src_in, float* dst, const int64_t* idx_all, const int64_t* it_cur,
                             int64_t* it_next, int64_t nb, int64_t Cin, int64_t hw, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(nb > 0 && Cin > 0 && hw > 0, "invalid shape");
        AIMET_REQUIRE(Cin * nb * hw < (int64_t(1) << 31), "batch too large for the channel-major gather");
        require_device_ptr(src_in, "src_in");
        require_device_ptr(dst, "dst");
        require_device_ptr(idx_all, "idx_all");
        require_device_ptr(it_cur, "it_cur");
        require_device_ptr(it_next, "it_next");
        const int64_t n = Cin * nb * hw;
        const bool vec  = hw % 4 == 0 && aligned16(src_in) && aligned16(dst);
        const int per   = vec ? 4 : 1;
        const unsigned blocks = (unsigned) ceil_div(n, (int64_t) kBlock * per);
        const FastDiv dhw((uint32_t) hw), dnb((uint32_t) nb);
        if (vec)
            adaround_gather_cm_kernel<4><<<blocks, kBlock, 0, as_stream(stream)>>>(
                src_in, dst, idx_all, it_cur, it_next, (uint32_t) nb, (uint32_t) Cin, (uint32_t) hw, (uint32_t) n, dhw, dnb);
        else
            adaround_gather_cm_kernel<1><<<blocks, kBlock, 0, as_stream(stream)>>>(
                src_in, dst, idx_all, it_cur, it_next, (uint32_t) nb, (uint32_t) Cin, (uint32_t) hw, (uint32_t) n, dhw, dnb);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_adaround_recon_grad_indexed_cm(const float* q, const float* out_data, const int64_t* idx_all,
                                         const int64_t* it_cur, float* g, int64_t nb, int64_t C, int64_t hw,
                                         const float* bias, int act, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(nb > 0 && C > 0 && hw > 0, "invalid shape");
        AIMET_REQUIRE(act >= 0 && act <= 2, "act must be 0 (none), 1 (ReLU) or 2 (ReLU6)");
        const int64_t n = nb * C * hw;
        AIMET_REQUIRE(n < (int64_t(1) << 31), "batch too large (>= 2^31 elements)");
        require_device_ptr(q, "quant_out");
        require_device_ptr(out_data, "out_data");
        require_device_ptr(idx_all, "idx_all");
        require_device_ptr(it_cur, "it_cur");
        require_device_ptr(g, "grad");
        if (bias)
            require_device_ptr(bias, "bias");
        const float scale = (float) (2.0 / (double) (nb * hw));   // as aimet_adaround_recon_grad_indexed
        ReconIdx r {out_data, idx_all, it_cur, bias, nb, C * hw, hw, C,
                    FastDiv((uint32_t) (C * hw)), FastDiv((uint32_t) hw), FastDiv((uint32_t) nb)};
        if (hw % 4 == 0 && aligned16(q) && aligned16(out_data) && aligned16(g))
            recon_grad_idx_cm_kernel<4><<<(unsigned) ceil_div(n, (int64_t) kBlock * 4), kBlock, 0, as_stream(stream)>>>(
                q, g, r, scale, act);
        else
            recon_grad_idx_cm_kernel<1><<<(unsigned) ceil_div(n, (int64_t) kBlock), kBlock, 0, as_stream(stream)>>>(
                q, g, r, scale, act);
        AIMET_LAUNCH_CHECK();
    });
}

int aimet_adaround_backward_adam_parts(const float* w, float* alpha, const float* grad_parts, int64_t nparts,
                                       int64_t part_kk, float* exp_avg, float* exp_avg_sq, int64_t outer, int64_t C, int64_t K,
                                       const float* delta, const float* offset, int32_t bw, const float* reg_beta_all,
                                       const int64_t* it_next, int64_t* it_cur, double lr, double beta1, double beta2,
                                       double eps, float* round_loss, float* wq_next, const float* bias_corr,
                                       void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(outer >= 0 && C > 0 && K >= 0, "invalid shape");
        if (bias_corr)
            require_device_ptr(bias_corr, "bias_corr");
        if (wq_next)
            require_device_ptr(wq_next, "wq_next");
        const int64_t n = outer * C * K;
        AIMET_REQUIRE(n > 0 && n < (int64_t(1) << 31), "AdaRound weight must have 1 .. 2^31-1 elements");
        require_device_ptr(w, "weight");
        require_device_ptr(alpha, "alpha");
        require_device_ptr(grad_parts, "grad");
        AIMET_REQUIRE(nparts >= 1 && nparts <= 65535, "nparts out of range");
        AIMET_REQUIRE(part_kk >= 0 && part_kk <= outer * C * K && (part_kk == 0 || (outer * C * K) % part_kk == 0),
                      "part_kk must be 0 or divide the weight's element count");
        const float* grad_wq = grad_parts;
        require_device_ptr(exp_avg, "exp_avg");
        require_device_ptr(exp_avg_sq, "exp_avg_sq");
        require_device_ptr(delta, "delta");
        require_device_ptr(offset, "offset");
        require_device_ptr(reg_beta_all, "reg_beta_all");
        require_device_ptr(it_next, "it_next");
        require_device_ptr(it_cur, "it_cur");
        AdaChannel map {FastDiv((uint32_t) (K > 0 ? K : 1)), FastDiv((uint32_t) C), (uint32_t) C};
        AdaParams p {(float) ((1ull << bw) - 1), 0.0f, 0.0f, 0.0f, 1, (uint32_t) (n - n % 32), round_loss != nullptr};
        AdamArgs a {lr, beta1, beta2, eps};
        // 4 elements per lane only for weights large enough to fill the chip that way: the per-element
        // chain (sigmoid, Sleef pow, Adam) is long, and a small layer's step is latency-bound, so
        // it takes one element per lane (4x the lanes; the same arithmetic per element)
        const bool vec = part_kk == 0 && n >= (int64_t(1) << 18) && (C == 1 || K % 4 == 0) && n % 4 == 0 && aligned16(w) && aligned16(alpha) &&
                         aligned16(grad_wq) && aligned16(exp_avg) && aligned16(exp_avg_sq) &&
                         (wq_next == nullptr || aligned16(wq_next));
        const int64_t items = vec ? n / 4 : n;
        int64_t blocks      = ceil_div(items, kBlock);
        blocks              = blocks < kAdaBwdGrid ? blocks : kAdaBwdGrid;
        hipStream_t st = as_stream(stream);
        LossFold lf(round_loss, (unsigned) blocks, st);
        auto launch = [&](auto kernel) {
            kernel<<<(unsigned) blocks, kBlock, 0, st>>>(w, alpha, grad_wq, exp_avg, exp_avg_sq, (uint32_t) n, map, delta,
                                                         offset, p, reg_beta_all, it_next, it_cur, a, round_loss,
                                                         wq_next, lf.part, lf.ticket, (uint32_t) nparts, bias_corr,
                                                         (uint32_t) part_kk);
        };
        const bool wl = round_loss != nullptr;
        if (!exact_pow())   // the fast pow: no scalar pow tail
        {
            if (vec)
                wl ? launch(adaround_bwd_adam_kernel<true, true, false, false>)
                   : launch(adaround_bwd_adam_kernel<true, false, false, false>);
            else
                wl ? launch(adaround_bwd_adam_kernel<false, true, true, false>)
                   : launch(adaround_bwd_adam_kernel<false, false, true, false>);
        }
        else if (vec && n % 32 == 0)   // no element in the scalar pow tail
            wl ? launch(adaround_bwd_adam_kernel<true, true, false, true>)
               : launch(adaround_bwd_adam_kernel<true, false, false, true>);
        else if (vec)
            wl ? launch(adaround_bwd_adam_kernel<true, true, true, true>)
               : launch(adaround_bwd_adam_kernel<true, false, true, true>);
        else
            wl ? launch(adaround_bwd_adam_kernel<false, true, true, true>)
               : launch(adaround_bwd_adam_kernel<false, false, true, true>);
        AIMET_LAUNCH_CHECK();
        lf.finish(0.0f, reg_beta_all, it_next, round_loss);
    });
}

int aimet_adaround_backward_adam(const float* w, float* alpha, const float* grad_wq, float* exp_avg, float* exp_avg_sq,
                                 int64_t outer, int64_t C, int64_t K, const float* delta, const float* offset,
                                 int32_t bw, const float* reg_beta_all, const int64_t* it_next, int64_t* it_cur,
                                 double lr, double beta1, double beta2, double eps, float* round_loss, float* wq_next,
                                 void* stream)
{
    return aimet_adaround_backward_adam_parts(w, alpha, grad_wq, 1, 0, exp_avg, exp_avg_sq, outer, C, K, delta, offset, bw,
                                              reg_beta_all, it_next, it_cur, lr, beta1, beta2, eps, round_loss, wq_next,
                                              nullptr, stream);
}

int aimet_adaround_set_exact_pow(int exact)
{
    return guarded([&] { exact_pow_flag().store(exact ? 1 : 0); });
}

int aimet_adaround_get_exact_pow(int* exact)
{
    return guarded([&] {
        AIMET_REQUIRE(exact != nullptr, "null argument");
        *exact = exact_pow() ? 1 : 0;
    });
}

int aimet_adaround_adam_bias_corrections(double beta1, double beta2, int64_t steps, float* bias_corr, void* stream)
{
    return guarded([&] {
        AIMET_REQUIRE(steps > 0 && steps < (int64_t(1) << 31), "steps out of range");
        require_device_ptr(bias_corr, "bias_corr");
        adam_bias_corr_kernel<<<(unsigned) ceil_div(steps, (int64_t) kBlock), kBlock, 0, as_stream(stream)>>>(
            beta1, beta2, steps, bias_corr);
        AIMET_LAUNCH_CHECK();
    });
}

}   // extern "C"
