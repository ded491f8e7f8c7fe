// Host-side f64 post-processing of the vocoder output, part of WaveRNN.generate
// (reference vocoder/models/fatchord_version.py:251-252 -> vocoder/audio.py:92-93):
// de_emphasis(x) = scipy.signal.lfilter([1], [1, -coef], x).
//
// scipy evaluates lfilter in direct form II transposed with b padded to len(a) and both
// vectors divided by a[0] (= 1 here, exact): per sample
//     y[n] = z + b0 * x[n];   z = x[n] * b1 - y[n] * a1     (b0 = 1, b1 = 0, a1 = -coef)
// The same expressions, evaluated in the same order without contraction (this file is built
// with -ffp-contract=off), give the same doubles bit for bit.
#include <cstddef>

#include "wavernn_mi355x.h"

extern "C" int wrnn_de_emphasis(const double* x, double* y, size_t n, double coef) {
    if (n && (!x || !y)) return WRNN_ERR_INVALID;
    const double b0 = 1.0, b1 = 0.0, a1 = -coef;
    double z = 0.0;
    for (size_t i = 0; i < n; ++i) {
        const double xn = x[i];
        const double yn = z + b0 * xn;
        z = xn * b1 - yn * a1;
        y[i] = yn;
    }
    return WRNN_OK;
}
