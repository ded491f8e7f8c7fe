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
#include <cstdint>

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

// Fused post-processing of categorical fold rows (fatchord_version.py:238-255 on batched
// labels): xfade_and_unfold (fatchord_version.py:342-404), decode_mu_law, de_emphasis and the
// final fade, in two passes over the labels with no intermediate full-length arrays.
//
// Unfolded layout (fold i starts at i * (target + overlap)): region 0 = fold 0's head, then per
// fold its untouched middle (target samples) followed by the region it shares with the next
// fold's head (the last fold's tail alone). numpy builds each sample as 0.0 + a (+ b), with
// a = sample * fade; the same sums in the same order are formed here.
//
// Pass 1 (wrnn_post_overlaps): the nf + 1 overlap regions, un-decoded, into regions
// [(nf + 1) * overlap]. The caller decodes them with the same numpy expression as the
// reference (so the transcendental is numpy's own), and builds `mid_lut` = the decoded value of
// every label (a middle sample is its label's value untouched).
// Pass 2 (wrnn_post_assemble): out[j], j < n_out, from mid_lut / regions, then the de-emphasis
// recurrence (if preemph) and out[n_out - fade_len + k] *= fade[k].
static int post_check(const int16_t* labels, int nf, int S, int overlap, int n_classes) {
    if (!labels || nf < 1 || overlap < 1 || S < 2 * overlap + 1 || n_classes < 2)
        return WRNN_ERR_INVALID;
    const size_t n = (size_t)nf * (size_t)S;
    for (size_t i = 0; i < n; ++i)
        if (labels[i] < 0 || labels[i] >= n_classes) return WRNN_ERR_INVALID;
    return WRNN_OK;
}

extern "C" int wrnn_post_overlaps(const int16_t* labels, int nf, int S, int overlap,
                                  const double* samp, int n_classes, const double* fade_in,
                                  const double* fade_out, double* regions) {
    const int rc = post_check(labels, nf, S, overlap, n_classes);
    if (rc) return rc;
    if (!samp || !fade_in || !fade_out || !regions) return WRNN_ERR_INVALID;
    for (int i = 0; i <= nf; ++i) {
        const int16_t* tail = i > 0 ? labels + (size_t)(i - 1) * S + (S - overlap) : nullptr;
        const int16_t* head = i < nf ? labels + (size_t)i * S : nullptr;
        double* r = regions + (size_t)i * overlap;
        for (int k = 0; k < overlap; ++k) {
            double v = 0.0;
            if (tail) v = v + samp[tail[k]] * fade_out[k];
            if (head) v = v + samp[head[k]] * fade_in[k];
            r[k] = v;
        }
    }
    return WRNN_OK;
}

extern "C" int wrnn_post_assemble(const int16_t* labels, int nf, int S, int overlap,
                                  const double* mid_lut, int n_classes, const double* regions,
                                  int preemph, double coef, const double* fade, size_t fade_len,
                                  double* out, size_t n_out) {
    const int rc = post_check(labels, nf, S, overlap, n_classes);
    if (rc) return rc;
    const int target = S - 2 * overlap;
    const size_t total = (size_t)nf * (size_t)(target + overlap) + (size_t)overlap;
    if (!mid_lut || !regions || !out || n_out > total || fade_len > n_out ||
        (fade_len && !fade))
        return WRNN_ERR_INVALID;
    size_t j = 0;
    for (int k = 0; k < overlap && j < n_out; ++k) out[j++] = regions[k];
    for (int i = 0; i < nf && j < n_out; ++i) {
        const int16_t* mid = labels + (size_t)i * S + overlap;
        for (int k = 0; k < target && j < n_out; ++k) out[j++] = mid_lut[mid[k]];
        const double* r = regions + (size_t)(i + 1) * overlap;
        for (int k = 0; k < overlap && j < n_out; ++k) out[j++] = r[k];
    }
    if (preemph) wrnn_de_emphasis(out, out, n_out, coef);
    double* tail = out + (n_out - fade_len);
    for (size_t k = 0; k < fade_len; ++k) tail[k] *= fade[k];
    return WRNN_OK;
}
