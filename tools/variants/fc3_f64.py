"""A/B variant: k_persist's fc3 logits from float64 sums of
the exact fp32 products, rounded once to fp32 after the bias -- l = RN(b + sum w x) -- instead of
the fp32 pairwise-by-lane sums. Source transform of kernels_persist.hip (dense instances; the
sparse ones keep the fp32 form); tools/build_patched.sh applies it to a copy of csrc/."""
import sys

path = sys.argv[1]
s = open(path).read()


def rep(old, new):
    global s
    assert s.count(old) == 1, old[:80]
    s = s.replace(old, new)


rep("""            float s0 = 0.f;
            auto fc3 = [&]() {
                if (!has_cls) return;""", """            float s0 = 0.f;
            double s0d = 0.0;
            auto fc3 = [&]() {
                if (!has_cls) return;
                double accd[NR];
#pragma unroll
                for (int r = 0; r < NR; ++r) accd[r] = 0.0;""")
rep("""#pragma unroll
                        for (int q = 0; q < 4; ++q) dot4(acc[r], wq[q], xq[q]);
                    }
                }
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const float t0 = row16_sum(hsum(acc[r]));
                    if (kc == r) s0 = t0;
                }""", """#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            if constexpr (SP) {
                                dot4(acc[r], wq[q], xq[q]);
                            } else {  // exact products, float64 sums
                                accd[r] = __builtin_fma((double)wq[q].x, (double)xq[q].x, accd[r]);
                                accd[r] = __builtin_fma((double)wq[q].y, (double)xq[q].y, accd[r]);
                                accd[r] = __builtin_fma((double)wq[q].z, (double)xq[q].z, accd[r]);
                                accd[r] = __builtin_fma((double)wq[q].w, (double)xq[q].w, accd[r]);
                            }
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    if constexpr (SP) {
                        const float t0 = row16_sum(hsum(acc[r]));
                        if (kc == r) s0 = t0;
                    } else {
                        double t = accd[r];
#pragma unroll
                        for (int o = 1; o < 16; o <<= 1) t += __shfl_xor(t, o, 16);
                        if (kc == r) s0d = t;
                    }
                }""")
rep("""                    l = p_add(s0, lds[L_BCLS + og]);""",
    """                    l = SP ? p_add(s0, lds[L_BCLS + og]) : (float)(s0d + (double)lds[L_BCLS + og]);""")
open(path, 'w').write(s)
