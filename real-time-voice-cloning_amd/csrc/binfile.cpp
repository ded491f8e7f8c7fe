// Reader of the libwavernn ".bin" weight format (host code, no device needed).
//
// Format written by the reference's vocoder/libwavernn/convert.py:38-58 (file header),
// :60-81 (1x4 block-compressed matrices), :83-156 (per-layer records), :303-351 (layer order);
// read by libwavernn/<variant>/src/wavernn.cpp:37-184. All integers are native int32; the
// arrays of a layer are fp32 ("elSize" 4) or IEEE binary16 ("elSize" 2, convert.py:12 "change
// to 2 for fp16"; widened to fp32 on load), the BatchNorm eps is always fp32; structs packed
// with Python's '@' (native) layout. (The reference's C++ reader accepts elSize 2 but freads
// the 2-byte elements straight into fp32 storage, wavernn.h:83 / wavernn.cpp:103, and its
// convert.py writes fp32 payloads whatever the header says, so no reference output exists for
// an fp16 file: here elSize 2 means what the header comment declares.)
//   header   int32 res_blocks, n_upsample, total_scale, pad
//   layer    int32 type (1 Conv1d, 2 Conv2d, 3 BatchNorm1d, 4 Linear, 5 GRU, 6 Stretch2d),
//            char name[64] (the module's repr), then the type's record:
//   Conv1d     int32 elSize, has_bias, in, out, k; f32 weight[out][in][k]; [f32 bias[out]]
//   Conv2d     int32 elSize, k; f32 weight[k]                       (1 x 1 x 1 x k kernels)
//   BatchNorm  int32 elSize, n; f32 eps; f32 weight[n], bias[n], running_mean[n], running_var[n]
//   Linear     int32 elSize, rows, cols; compressed weight; f32 bias[rows]
//   GRU        int32 elSize, hidden, input; compressed W_ir, W_iz, W_in, W_hr, W_hz, W_hn;
//              f32 b_ir, b_iz, b_in, b_hr, b_hz, b_hn [hidden each]
//   Stretch2d  int32 x_scale, y_scale
//   compressed int32 nw; f32 w[nw]; int32 ni; uint8 idx[ni]: for every row the indices of its
//              4-column groups holding a non-zero (in order) then 255, plus one trailing 255;
//              w holds those groups' 4 values row by row (Pruner's 1x4 block sparsity,
//              vocoder/pruner.py). Dense matrices are the special case "every group present".
// Emits every tensor under its PyTorch state-dict name and layout (gate order r, z, n), so a
// .bin file loads through the same path as a checkpoint.
#include "wavernn_mi355x.h"

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

extern "C" int wrnn_internal_fail(int code, const char* msg);  // runtime.hip

namespace {

int bfail(int code, const std::string& msg) { return wrnn_internal_fail(code, msg.c_str()); }

constexpr int kGroup = 4;  // hparams sparse_group (config/hparams.py) used by convert.py

// IEEE binary16 -> binary32 (exact: every half is a float)
float half_to_float(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu, bits;
    if (e == 0x1f) {
        bits = sign | 0x7f800000u | (m << 13);  // inf / nan
    } else if (e != 0) {
        bits = sign | ((e + 112u) << 23) | (m << 13);
    } else if (m == 0) {
        bits = sign;
    } else {  // subnormal: normalise
        int sh = 0;
        while (!(m & 0x400u)) {
            m <<= 1;
            ++sh;
        }
        bits = sign | ((uint32_t)(113 - sh) << 23) | ((m & 0x3ffu) << 13);
    }
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

struct Reader {
    const uint8_t* p;
    size_t n, off = 0;
    int es = 4;  // element size of the current layer's arrays
    std::string err;
    bool take(void* dst, size_t k) {
        if (!err.empty()) return false;
        if (k > n - off) {
            err = "truncated file at byte " + std::to_string(off);
            return false;
        }
        std::memcpy(dst, p + off, k);
        off += k;
        return true;
    }
    int32_t i32() {
        int32_t v = 0;
        take(&v, 4);
        return v;
    }
    float f32() {
        float v = 0;
        take(&v, 4);
        return v;
    }
    std::vector<float> floats(int64_t k) {
        std::vector<float> v;
        if (!err.empty()) return v;
        if (k < 0 || (uint64_t)k * es > n - off) {
            err = "bad array length " + std::to_string(k) + " at byte " + std::to_string(off);
            return v;
        }
        v.resize((size_t)k);
        if (es == 4) {
            take(v.data(), (size_t)k * 4);
        } else {
            for (int64_t i = 0; i < k; ++i) {
                uint16_t h;
                std::memcpy(&h, p + off + 2 * (size_t)i, 2);
                v[(size_t)i] = half_to_float(h);
            }
            off += (size_t)k * 2;
        }
        return v;
    }
};

struct Emitter {
    wrnn_tensor_fn fn;
    void* user;
    int rc = WRNN_OK;
    void operator()(const std::string& name, const std::vector<float>& d, std::vector<int64_t> shape) {
        int64_t count = 1;
        for (int64_t v : shape) count *= v;
        if (rc || (int64_t)d.size() != count) return;  // short read: the reader has the error
        rc = fn(user, name.c_str(), d.data(), shape.data(), (int)shape.size());
    }
};

enum LayerType { L_CONV1D = 1, L_CONV2D = 2, L_BN = 3, L_LINEAR = 4, L_GRU = 5, L_STRETCH = 6 };

bool layer_header(Reader& r, int want) {
    const int t = r.i32();
    char name[64];
    r.take(name, 64);
    if (!r.err.empty()) return false;
    if (t != want) {
        static const char* names[] = {"?", "Conv1d", "Conv2d", "BatchNorm1d", "Linear", "GRU", "Stretch2d"};
        r.err = std::string("expected a ") + names[want] + " layer at byte " + std::to_string(r.off - 68) +
                ", found type " + std::to_string(t);
        return false;
    }
    return true;
}

bool el_size(Reader& r) {  // wavernn.cpp:98 `assert(header.elSize==4 or header.elSize==2)`
    const int e = r.i32();
    if (r.err.empty() && e != 4 && e != 2)
        r.err = "elSize " + std::to_string(e) + " at byte " + std::to_string(r.off - 4) + " (4 = fp32, 2 = fp16)";
    r.es = e == 2 ? 2 : 4;
    return r.err.empty();
}

// 1x4 block-compressed (rows, cols) matrix -> dense row-major
std::vector<float> compressed(Reader& r, int rows, int cols) {
    std::vector<float> out;
    const int nw = r.i32();
    std::vector<float> w = r.floats(nw);
    const int ni = r.i32();
    if (!r.err.empty()) return out;
    if (ni < 0 || (size_t)ni > r.n - r.off) {
        r.err = "bad index length " + std::to_string(ni);
        return out;
    }
    const uint8_t* idx = r.p + r.off;
    r.off += (size_t)ni;
    if (cols % kGroup || cols / kGroup > 255) {
        r.err = "matrix width " + std::to_string(cols) + " is not a multiple of 4 below 1024";
        return out;
    }
    out.assign((size_t)rows * cols, 0.f);
    size_t ip = 0, wp = 0;
    for (int row = 0; row < rows; ++row) {
        int last = -1;
        while (true) {
            if (ip >= (size_t)ni) {
                r.err = "index stream ends inside row " + std::to_string(row);
                return out;
            }
            const int g = idx[ip++];
            if (g == 255) break;
            if (g <= last || g >= cols / kGroup || wp + kGroup > w.size()) {
                r.err = "bad group index " + std::to_string(g) + " in row " + std::to_string(row);
                return out;
            }
            last = g;
            std::memcpy(&out[(size_t)row * cols + (size_t)g * kGroup], &w[wp], kGroup * sizeof(float));
            wp += kGroup;
        }
    }
    // convert.py appends one more 255 for a row past the end
    if (ip >= (size_t)ni || idx[ip] != 255 || ip + 1 != (size_t)ni || wp != w.size())
        r.err = "index / weight stream lengths do not match the matrix";
    return out;
}

void conv1d(Reader& r, Emitter& E, const std::string& pfx, int in, int out, int k, bool bias) {
    if (!layer_header(r, L_CONV1D) || !el_size(r)) return;
    const int hb = r.i32(), ci = r.i32(), co = r.i32(), kk = r.i32();
    if (!r.err.empty()) return;
    if (ci != in || co != out || kk != k || (hb != 0) != bias) {
        r.err = pfx + ": Conv1d(" + std::to_string(ci) + ", " + std::to_string(co) + ", k=" + std::to_string(kk) +
                ") does not match the model";
        return;
    }
    E(pfx + ".weight", r.floats((int64_t)out * in * k), {out, in, k});
    if (bias) E(pfx + ".bias", r.floats(out), {out});
}

void batchnorm(Reader& r, Emitter& E, const std::string& pfx, int n) {
    if (!layer_header(r, L_BN) || !el_size(r)) return;
    const int nf = r.i32();
    const float eps = r.f32();
    if (!r.err.empty()) return;
    if (nf != n || eps != 1e-5f) {
        r.err = pfx + ": BatchNorm1d(" + std::to_string(nf) + ", eps) does not match the model (eps 1e-5)";
        return;
    }
    for (const char* f : {".weight", ".bias", ".running_mean", ".running_var"}) E(pfx + f, r.floats(n), {n});
}

void linear(Reader& r, Emitter& E, const std::string& pfx, int in, int out) {
    if (!layer_header(r, L_LINEAR) || !el_size(r)) return;
    const int rows = r.i32(), cols = r.i32();
    if (!r.err.empty()) return;
    if (rows != out || cols != in) {
        r.err = pfx + ": Linear(" + std::to_string(cols) + ", " + std::to_string(rows) + ") does not match the model";
        return;
    }
    std::vector<float> W = compressed(r, rows, cols);
    E(pfx + ".weight", W, {rows, cols});
    E(pfx + ".bias", r.floats(rows), {rows});
}

void gru(Reader& r, Emitter& E, const std::string& pfx, int in, int H) {
    if (!layer_header(r, L_GRU) || !el_size(r)) return;
    const int hid = r.i32(), inp = r.i32();
    if (!r.err.empty()) return;
    if (hid != H || inp != in) {
        r.err = pfx + ": GRU(" + std::to_string(inp) + ", " + std::to_string(hid) + ") does not match the model";
        return;
    }
    std::vector<float> wih, whh, bih, bhh;
    for (int j = 0; j < 3; ++j) {
        std::vector<float> m = compressed(r, H, in);
        wih.insert(wih.end(), m.begin(), m.end());
    }
    for (int j = 0; j < 3; ++j) {
        std::vector<float> m = compressed(r, H, H);
        whh.insert(whh.end(), m.begin(), m.end());
    }
    for (int j = 0; j < 3; ++j) {
        std::vector<float> b = r.floats(H);
        bih.insert(bih.end(), b.begin(), b.end());
    }
    for (int j = 0; j < 3; ++j) {
        std::vector<float> b = r.floats(H);
        bhh.insert(bhh.end(), b.begin(), b.end());
    }
    if (!r.err.empty()) return;
    E(pfx + ".weight_ih_l0", wih, {3 * H, in});
    E(pfx + ".weight_hh_l0", whh, {3 * H, H});
    E(pfx + ".bias_ih_l0", bih, {3 * H});
    E(pfx + ".bias_hh_l0", bhh, {3 * H});
}

void stretch(Reader& r, int xs, int ys) {
    if (!layer_header(r, L_STRETCH)) return;
    const int x = r.i32(), y = r.i32();
    if (r.err.empty() && (x != xs || y != ys))
        r.err = "Stretch2d(" + std::to_string(x) + ", " + std::to_string(y) + ") does not match the model";
}

}  // namespace

extern "C" int wrnn_bin_read(const void* data, size_t bytes, const wrnn_config* cfg, wrnn_tensor_fn fn,
                             void* user) {
    if (!data || !cfg || !fn) return bfail(WRNN_ERR_INVALID, "null argument");
    // the topology comes from the caller: bound what indexes or shifts below
    if (cfg->n_upsample < 1 || cfg->n_upsample > 4 || (cfg->mode == WRNN_MODE_RAW && (cfg->bits < 2 || cfg->bits > 12)) ||
        cfg->res_blocks < 0 || cfg->res_blocks > 64 || cfg->rnn_dims <= 0 || cfg->fc_dims <= 0 ||
        cfg->compute_dims <= 0 || cfg->res_out_dims <= 0 || cfg->feat_dims <= 0 || cfg->pad < 0)
        return bfail(WRNN_ERR_INVALID, "libwavernn .bin: invalid model configuration");
    Reader r{static_cast<const uint8_t*>(data), bytes};
    Emitter E{fn, user};
    const int res_blocks = r.i32(), n_up = r.i32(), total_scale = r.i32(), pad = r.i32();
    if (!r.err.empty()) return bfail(WRNN_ERR_INVALID, "Cannot open file.");
    if (res_blocks != cfg->res_blocks || n_up != cfg->n_upsample || total_scale != cfg->hop_length ||
        pad != cfg->pad)
        return bfail(
            WRNN_ERR_INVALID, "file header (res_blocks " + std::to_string(res_blocks) + ", upsample stages " +
                                  std::to_string(n_up) + ", scale " + std::to_string(total_scale) + ", pad " +
                                  std::to_string(pad) + ") does not match the model configuration");
    const int C = cfg->compute_dims, R = cfg->res_out_dims, F0 = cfg->feat_dims, H = cfg->rnn_dims,
              Fc = cfg->fc_dims, k_in = 2 * cfg->pad + 1;
    const int n = cfg->mode == WRNN_MODE_RAW ? (1 << cfg->bits) : cfg->mode == WRNN_MODE_BETA ? 2 : 30;
    // MelResNet (convert.py:310-320)
    conv1d(r, E, "upsample.resnet.conv_in", F0, C, k_in, false);
    batchnorm(r, E, "upsample.resnet.batch_norm", C);
    for (int i = 0; i < res_blocks && r.err.empty(); ++i) {
        const std::string p = "upsample.resnet.layers." + std::to_string(i);
        conv1d(r, E, p + ".conv1", C, C, 1, false);
        batchnorm(r, E, p + ".batch_norm1", C);
        conv1d(r, E, p + ".conv2", C, C, 1, false);
        batchnorm(r, E, p + ".batch_norm2", C);
    }
    conv1d(r, E, "upsample.resnet.conv_out", C, R, 1, true);
    stretch(r, total_scale, 1);
    // upsample stages: Stretch2d(s, 1), Conv2d(1, 1, (1, 2s+1)) (convert.py:322-325)
    for (int j = 0; j < n_up && r.err.empty(); ++j) {
        const int s = cfg->upsample_factors[j];
        stretch(r, s, 1);
        if (!layer_header(r, L_CONV2D) || !el_size(r)) break;
        const int k = r.i32();
        if (r.err.empty() && k != 2 * s + 1) {
            r.err = "upsample kernel " + std::to_string(k) + " != 2 * scale + 1";
            break;
        }
        E("upsample.up_layers." + std::to_string(2 * j + 1) + ".weight", r.floats(k), {1, 1, 1, k});
    }
    // main network (convert.py:327-351)
    const int A = R / (cfg->model_type == WRNN_MODEL_GENEING ? 2 : 4);
    linear(r, E, "I", F0 + A, H);
    if (cfg->model_type == WRNN_MODEL_GENEING) {  // convert.py:336-340
        gru(r, E, "rnn1", H, H);
        linear(r, E, "fc1", H + A, Fc);
        linear(r, E, "fc3", Fc, n);
    } else if (cfg->model_type == WRNN_MODEL_FATCHORD) {
        gru(r, E, "rnn1", H, H);
        gru(r, E, "rnn2", H + A, H);
        linear(r, E, "fc1", H + A, Fc);
        linear(r, E, "fc2", Fc + A, Fc);
        linear(r, E, "fc3", Fc, n);
    } else if (cfg->model_type == WRNN_MODEL_RUNTIMERACER) {
        gru(r, E, "rnn1", H, H);
        gru(r, E, "rnn2", H, H);
        gru(r, E, "rnn3", H + A, H);
        gru(r, E, "rnn4", H, H);
        linear(r, E, "fc1", H + A, Fc);
        linear(r, E, "fc2", Fc, Fc);
        linear(r, E, "fc3", Fc + A, Fc);
        linear(r, E, "fc4", Fc, Fc);
        linear(r, E, "fc5", Fc, n);
    } else {
        return bfail(WRNN_ERR_INVALID, "Invalid model type " + std::to_string(cfg->model_type));
    }
    if (r.err.empty() && r.off != r.n) r.err = std::to_string(r.n - r.off) + " trailing bytes after the last layer";
    if (!r.err.empty()) return bfail(WRNN_ERR_INVALID, "libwavernn .bin: " + r.err);
    if (E.rc) return E.rc;
    return WRNN_OK;
}
