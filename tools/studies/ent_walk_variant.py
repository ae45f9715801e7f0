"""Writes a study copy of entropy_search.hip whose asymmetric window list comes from a one-lane walk
with the next step's bins loaded ahead and the zero-representability tests precomputed per bin
(the reference's decisions), for timing against entropy::windows. usage: ent_walk_variant.py SRC OUT"""
import sys

WALK = '''// study: entropy::windows for one side-choosing walk by one lane (prefetched bins, tests from zr)
__device__ int windows_walk(const double* hist, const uint8_t* zr, short* wa, short* wb)
{
    using namespace entropy;
    int a = 0, b = kBins - 1, n = 0;
    double ha = hist[a], ha1 = hist[a + 1], hb = hist[b], hb1 = hist[b - 1];
    while (b - a + 1 >= kLevels)
    {
        wa[n] = (short) a;
        wb[n] = (short) b;
        ++n;
        const double ha2 = hist[a + 2], ha3 = hist[a + 3], hb2 = hist[b - 2], hb3 = hist[b - 3];
        const uint32_t za1 = zr[a + 1], za2 = zr[a + 2], zb = zr[b], zb1 = zr[b - 1];
        const double loss0 = ha + hb, loss1 = ha + ha1, loss2 = hb + hb1;
        int k = 0;
        if (loss1 < loss0)
            k = 1;
        if (loss2 < (k == 1 ? loss1 : loss0))
            k = 2;
        if ((k == 0 && (za1 & 1u)) || (k == 1 && (za2 & 1u)))
            k = 2;
        else if ((k == 0 && (zb & 2u)) || (k == 2 && (zb1 & 2u)))
            k = 1;
        if (k == 0)
        {
            ++a;
            --b;
            ha  = ha1;
            ha1 = ha2;
            hb  = hb1;
            hb1 = hb2;
        }
        else if (k == 1)
        {
            a += 2;
            ha  = ha2;
            ha1 = ha3;
        }
        else
        {
            b -= 2;
            hb  = hb2;
            hb1 = hb3;
        }
    }
    return n;
}

'''


def main():
    s = open(sys.argv[1]).read()

    def rep(a, b):
        nonlocal s
        assert s.count(a) == 1, a[:60]
        s = s.replace(a, b)
    rep("__global__ __launch_bounds__(kEntBlock)", WALK + "__global__ __launch_bounds__(kEntBlock)")
    rep("    __shared__ int s_n, s_rule, s_integral;",
        "    __shared__ int s_n, s_rule, s_integral;\n    __shared__ uint8_t s_zr[entropy::kBins];")
    rep('''                    wb[n] = (short) (entropy::kBins - 1 - n);
                }
            }
            if (t == 0)''', '''                    wb[n] = (short) (entropy::kBins - 1 - n);
                }
            }
            else
            {
                const double w = (dhi - dlo) / (double) entropy::kBins;
                for (int k = t; k < entropy::kBins; k += kEntBlock)
                {
                    const double e = dlo + (double) k * w;
                    s_zr[k]        = (uint8_t) ((e > 0 ? 1u : 0u) | (e < 0 ? 2u : 0u));
                }
                __syncthreads();
            }
            if (t == 0)''')
    rep(": entropy::windows(hist, dlo, (dhi - dlo) / (double) entropy::kBins, false, wa, wb);",
        ": windows_walk(hist, s_zr, wa, wb);")
    open(sys.argv[2], "w").write(s)


if __name__ == "__main__":
    main()
