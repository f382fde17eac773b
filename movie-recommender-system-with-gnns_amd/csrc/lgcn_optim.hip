// Fused training-step tail for gfx950: global grad-norm clip + dense Adam in two HBM passes.
//
// Reference utils/train_test.py:95-96 runs
//     torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1)
//     optimizer.step()            # optim.Adam(lr=1e-3) (:236), foreach implementation
// over the two dense tables (user_embedding.weight [U,d], item_embedding.weight [I,d]). PyTorch does
// that as ~20 multi-tensor launches per step (norms, stack, mul, lerp, mul, addcmul, sqrt, div,
// add, addcdiv), several of which materialise temporaries. Here:
//   pass 1 (k_sqnorm_partial + k_norm_finish): deterministic two-stage sum of squares ->
//           total_norm, clip_coef = min(max_norm / (total_norm + 1e-6), 1)   (on device, no sync)
//   pass 2 (k_adam): per element  g *= coef;  m = m + (1-b1)(g - m);  v = b2 v + (1-b2) g g;
//           p += step_size * m / (sqrt(v) / sqrt(bc2) + eps)        (torch's Adam, no decay)
// reading p, g, m, v once and writing p, m, v (+ g when the caller wants the clipped grad kept).
// Results agree with the PyTorch sequence to fp32 rounding (different reduction order), not bitwise.

#include <algorithm>

#include "lgcn_common.h"

using namespace lgcn;

namespace {

constexpr int kMaxTensors = 8;
constexpr int kNormBlocks = 1024;

struct TensorList {
    float* param[kMaxTensors];
    float* grad[kMaxTensors];
    float* exp_avg[kMaxTensors];
    float* exp_avg_sq[kMaxTensors];
    int64_t numel[kMaxTensors];
    int64_t offset[kMaxTensors + 1];  // prefix sums of numel
    int n;
};

__global__ __launch_bounds__(kBlock) void k_sqnorm_partial(TensorList t, float* __restrict__ partial) {
    __shared__ float red[kBlock / 64];
    float acc = 0.f;
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    // per tensor: float4 sweep of the aligned body, scalar tail (fixed assignment -> deterministic)
    for (int k = 0; k < t.n; ++k) {
        const float* G = t.grad[k];
        const int64_t n = t.numel[k];
        int64_t done = 0;
        if ((reinterpret_cast<uintptr_t>(G) & 15u) == 0) {
            const int64_t n4 = n / 4;
            const float4* G4 = reinterpret_cast<const float4*>(G);
            for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
                const float4 g = G4[i];
                acc += g.x * g.x + g.y * g.y + g.z * g.z + g.w * g.w;
            }
            done = n4 * 4;
        }
        for (int64_t i = done + int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) acc += G[i] * G[i];
    }
    // fixed-order wave + block reduction
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int w = 0; w < kBlock / 64; ++w) s += red[w];
        partial[blockIdx.x] = s;
    }
}

__global__ __launch_bounds__(kBlock) void k_norm_finish(const float* __restrict__ partial, int nparts,
                                                        float max_norm, float* __restrict__ out) {
    __shared__ float red[kBlock / 64];
    float acc = 0.f;
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += partial[i];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float s = 0.f;
        for (int w = 0; w < kBlock / 64; ++w) s += red[w];
        const float norm = sqrtf(s);
        const float coef = max_norm / (norm + 1e-6f);
        out[0] = norm;
        out[1] = coef < 1.0f ? coef : 1.0f;
    }
}

struct AdamScalars {
    float one_minus_beta1;
    float beta2;
    float one_minus_beta2;
    float step_size;  // -lr / (1 - beta1^t)
    float bc2_sqrt;   // sqrt(1 - beta2^t)
    float eps;
    int write_grad;
};

__device__ __forceinline__ void adam_elem(float& p, float& g, float& m, float& v, float coef, const AdamScalars& s) {
    g = g * coef;
    m = m + s.one_minus_beta1 * (g - m);
    v = v * s.beta2;
    v = v + s.one_minus_beta2 * (g * g);
    const float denom = sqrtf(v) / s.bc2_sqrt + s.eps;
    p = p + s.step_size * (m / denom);
}

// Device-side step counter and bias corrections (capturable Adam: a replayed hipGraph advances
// the step on the device). Same double-precision formulas torch evaluates on the host.
__global__ void k_adam_prologue(double* __restrict__ step, float lr, double beta1, double beta2,
                                float* __restrict__ scalars) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const double t = step[0] + 1.0;
        step[0] = t;
        const double bc1 = 1.0 - pow(beta1, t);
        const double bc2 = 1.0 - pow(beta2, t);
        scalars[0] = static_cast<float>(-(static_cast<double>(lr) / bc1));
        scalars[1] = static_cast<float>(sqrt(bc2));
    }
}

// One block-stride sweep per tensor, float4 where the tensor is 16-byte aligned and long enough.
__global__ __launch_bounds__(kBlock) void k_adam(TensorList t, AdamScalars s, const float* __restrict__ clip,
                                                 const float* __restrict__ dev_scalars) {
    const float coef = clip ? clip[1] : 1.0f;
    if (dev_scalars) {
        s.step_size = dev_scalars[0];
        s.bc2_sqrt = dev_scalars[1];
    }
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int k = 0; k < t.n; ++k) {
        float* P = t.param[k];
        float* G = t.grad[k];
        float* M = t.exp_avg[k];
        float* V = t.exp_avg_sq[k];
        const int64_t n = t.numel[k];
        const bool vec = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(G) |
                           reinterpret_cast<uintptr_t>(M) | reinterpret_cast<uintptr_t>(V)) & 15u) == 0;
        int64_t done = 0;
        if (vec) {
            const int64_t n4 = n / 4;
            for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
                float4 p = reinterpret_cast<float4*>(P)[i];
                float4 g = reinterpret_cast<float4*>(G)[i];
                float4 m = reinterpret_cast<float4*>(M)[i];
                float4 v = reinterpret_cast<float4*>(V)[i];
                adam_elem(p.x, g.x, m.x, v.x, coef, s);
                adam_elem(p.y, g.y, m.y, v.y, coef, s);
                adam_elem(p.z, g.z, m.z, v.z, coef, s);
                adam_elem(p.w, g.w, m.w, v.w, coef, s);
                reinterpret_cast<float4*>(P)[i] = p;
                reinterpret_cast<float4*>(M)[i] = m;
                reinterpret_cast<float4*>(V)[i] = v;
                if (s.write_grad) reinterpret_cast<float4*>(G)[i] = g;
            }
            done = n4 * 4;
        }
        for (int64_t i = done + int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
            float p = P[i], g = G[i], m = M[i], v = V[i];
            adam_elem(p, g, m, v, coef, s);
            P[i] = p;
            M[i] = m;
            V[i] = v;
            if (s.write_grad) G[i] = g;
        }
    }
}

int make_list(const lgcn_adam_tensor_t* ts, int n, TensorList& t, bool need_state) {
    if (!ts || n < 1 || n > kMaxTensors) return fail(LGCN_E_ARG, "lgcn optim: 1..%d tensors, got %d", kMaxTensors, n);
    t.n = n;
    t.offset[0] = 0;
    for (int k = 0; k < kMaxTensors; ++k) {
        const bool live = k < n;
        t.param[k] = live ? ts[k].param : nullptr;
        t.grad[k] = live ? ts[k].grad : nullptr;
        t.exp_avg[k] = live ? ts[k].exp_avg : nullptr;
        t.exp_avg_sq[k] = live ? ts[k].exp_avg_sq : nullptr;
        t.numel[k] = live ? ts[k].numel : 0;
        if (live) {
            if (ts[k].numel < 0 || (ts[k].numel > 0 && !ts[k].grad))
                return fail(LGCN_E_ARG, "lgcn optim: tensor %d has no grad", k);
            if (need_state && ts[k].numel > 0 && (!ts[k].param || !ts[k].exp_avg || !ts[k].exp_avg_sq))
                return fail(LGCN_E_ARG, "lgcn optim: tensor %d lacks param/state", k);
        }
        t.offset[k + 1] = t.offset[k] + t.numel[k];
    }
    return LGCN_OK;
}

}  // namespace

extern "C" {

int lgcn_grad_norm_workspace_floats(void) { return kNormBlocks; }

int lgcn_grad_norm(const lgcn_adam_tensor_t* tensors, int32_t n, float max_norm, float* ws, float* out,
                   lgcn_stream_t stream) {
    TensorList t;
    if (int rc = make_list(tensors, n, t, false)) return rc;
    if (!ws || !out) return fail(LGCN_E_ARG, "lgcn_grad_norm: null workspace/out");
    hipStream_t s = as_stream(stream);
    const int64_t total = t.offset[t.n];
    const unsigned blocks = static_cast<unsigned>(std::min<int64_t>(kNormBlocks, std::max<int64_t>(1, (total + kBlock - 1) / kBlock)));
    k_sqnorm_partial<<<blocks, kBlock, 0, s>>>(t, ws);
    if (int rc = check_launch("k_sqnorm_partial")) return rc;
    k_norm_finish<<<1, kBlock, 0, s>>>(ws, static_cast<int>(blocks), max_norm, out);
    return check_launch("k_norm_finish");
}

int lgcn_adam_prologue(double* step, float lr, double beta1, double beta2, float* scalars, lgcn_stream_t stream) {
    if (!step || !scalars) return fail(LGCN_E_ARG, "lgcn_adam_prologue: null pointer");
    k_adam_prologue<<<1, 64, 0, as_stream(stream)>>>(step, lr, beta1, beta2, scalars);
    return check_launch("k_adam_prologue");
}

int lgcn_adam_step(const lgcn_adam_tensor_t* tensors, int32_t n, float one_minus_beta1, float beta2,
                   float one_minus_beta2, float eps, float step_size, float bc2_sqrt, const float* clip,
                   const float* dev_scalars, int32_t write_grad, lgcn_stream_t stream) {
    TensorList t;
    if (int rc = make_list(tensors, n, t, true)) return rc;
    AdamScalars sc{one_minus_beta1, beta2, one_minus_beta2, step_size, bc2_sqrt, eps, write_grad};
    const int64_t total = t.offset[t.n];
    if (total == 0) return LGCN_OK;
    const unsigned blocks = grid_for(total / 4 + 1, kBlock, 8192);
    k_adam<<<blocks, kBlock, 0, as_stream(stream)>>>(t, sc, clip, dev_scalars);
    return check_launch("k_adam");
}

}  // extern "C"
