// Persistent decode step for gfx950: ONE launch runs n_steps whole decode steps (every
// layer's five phases, the lm_head, the sampler and the next token's embedding), replacing
// the 142 launches per token of the graph path (llm_kernels.hip) for the same
// llama_decode + sampler work (test-to-speech.cpp:161-190).
//
// Why: the graph path's per-layer launches stream 2.7-14 MB each and are latency bound
// (profiles/r01_v6_step_timeline.txt: ~1.4 us boundary + ~1 us dispatch / first-load
// latency + prologue per launch). Inside one launch a phase hand-off costs about what a
// boundary does (tools/micro/barrier_probe.hip: 2.4 vs 2.05 us for the same publish +
// read-back), but a workgroup can issue the NEXT phase's weight loads before it waits:
// weights never depend on the step's data, so every phase starts with its weights in
// registers (K/V cache rows likewise for the attention phase).
//
// Geometry: one 512-thread workgroup per CU, all resident (grid = CU count, > 80 KB of LDS
// keeps it at one per CU). Wave 0 is the hand-off wave: it arrives, polls, and stages the
// next phase's inputs into LDS; waves 1-7 own the matvec rows and issue their prefetch while
// wave 0 polls (a wave with weight loads in flight cannot poll: vmcnt retires in order).
// All 8 waves run the activation prologues (RMSNorm, re-quantization, attention merge).
//
// Hand-off protocol (cdna_hip_programming.md Guideline 16, R1 with sc1 loads): every value
// another workgroup reads is stored write-through (sc1) and read by sc1 loads; each wave
// drains its stores (s_waitcnt vmcnt(0)) before a workgroup barrier, after which ONE lane
// adds to the workgroup's counter shard (8 shards, one per XCD by blockIdx % 8); wave 0 polls
// the 8 shards (sc1) until they sum to G * epoch, stages inputs, then a workgroup barrier
// releases the other waves. Spins are bounded: a timeout sets the error word, which every
// poller also watches, so the grid always drains.
//
// Arithmetic is the graph path's, function for function (same quantizers, same integer
// block dots, same attention chunk decomposition and merge order), so the two paths agree
// bit for bit (tests/test_llm_gpu.py::test_persistent_matches_graph).
#include <hip/hip_runtime.h>

// an opaque copy of threadIdx.x per use (see llm_device.h)
__device__ __forceinline__ unsigned mio_opaque_tid() {
    unsigned t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}
#define MIO_TIDX mio_opaque_tid()
#include "llm_device.h"

#include <algorithm>

#pragma clang fp contract(off)

namespace mio {
namespace {

constexpr int PW = MW - 1;  // row waves (1..7); wave 0 is the hand-off wave
constexpr int kSpinLimit = 1 << 22;
constexpr int AUX_SC1 = 16;  // buffer-op cache bits: sc1 (device-coherent, write-through)

__device__ __forceinline__ void st_sc1(float *p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int AUX>
__device__ __forceinline__ float4 ld4(const float *base, uint32_t bytes, uint32_t off) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base, bytes), off, 0, AUX);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// One wave copies n floats (n % 4 == 0) from global to LDS, B 16-byte loads per lane in
// flight; aux = AUX_SC1 for handed-off data, 0 for constant data (norm weights).
template <int B, int AUX>
__device__ void stage(float *dst, const float *src, int n) {
    const int lane = MIO_TIDX & 63, nv = n >> 2;
    for (int v0 = 0; v0 < nv; v0 += 64 * B) {
        float4 t[B];
#pragma unroll
        for (int j = 0; j < B; ++j) t[j] = ld4<AUX>(src, (uint32_t)n * 4, (uint32_t)(v0 + j * 64 + lane) * 16);
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const int v = v0 + j * 64 + lane;
            if (v < nv) *reinterpret_cast<float4 *>(dst + 4 * v) = t[j];
        }
    }
}

// RMSNorm + re-quantization of an LDS-resident activation (x and norm weight staged by
// wave 0): the graph path's rmsnorm_quant / plain_quant on the same per-thread slices.
template <int XV>
__device__ void lds_xregs(const float *x, const float *w, int K, XRegs<XV> &xr) {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
        const int e = (MIO_TIDX + i * MT) * 4;
        xr.v[i] = e < K ? *reinterpret_cast<const float4 *>(x + e) : make_float4(0.f, 0.f, 0.f, 0.f);
        xr.w[i] = (w && e < K) ? *reinterpret_cast<const float4 *>(w + e) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// merge_attention (llm_device.h) with every partial-record load sc1 (records written by
// other workgroups in the attention phase of this launch)
template <int NP>
__device__ void merge_attention_sc1(const LlmDims &d, const float *part, int nch, int K, bool kquant, const Smem &s) {
    const int hd = d.hd, rec = part_rec(hd);
    const uint32_t pbytes = (uint32_t)((size_t)d.n_head * d.max_splits * rec * 4);
    const auto rp = rsrc(part, pbytes);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int e = (MIO_TIDX + i * MT) * 4;
        if (e < K) {
            const int h = e / hd, dd = e - h * hd;
            const uint32_t base = (uint32_t)((size_t)h * d.max_splits * rec) * 4;
            float M = -INFINITY, L = 0.0f;
            float4 O = make_float4(0.f, 0.f, 0.f, 0.f);
            constexpr int CB = 8;
            for (int c0 = 0; c0 < nch; c0 += CB) {
                float2 ml[CB];
                float4 oc[CB];
#pragma unroll
                for (int j = 0; j < CB; ++j) {
                    const int c = c0 + j;
                    if (c < nch) {
                        const uint32_t r = base + (uint32_t)(c * rec) * 4;
                        const auto m2 = __builtin_amdgcn_raw_buffer_load_b64(rp, r + hd * 4, 0, AUX_SC1);
                        ml[j] = make_float2(__uint_as_float(m2[0]), __uint_as_float(m2[1]));
                        const u32x4 o4 = __builtin_amdgcn_raw_buffer_load_b128(rp, r + dd * 4, 0, AUX_SC1);
                        oc[j] = make_float4(__uint_as_float(o4.x), __uint_as_float(o4.y), __uint_as_float(o4.z),
                                            __uint_as_float(o4.w));
                    } else {
                        ml[j] = make_float2(-INFINITY, 0.0f);
                        oc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                }
                float mb = M;
#pragma unroll
                for (int j = 0; j < CB; ++j) mb = fmaxf(mb, ml[j].x);
                const float a = M == -INFINITY ? 0.0f : expf(M - mb);
                L *= a;
                O.x *= a, O.y *= a, O.z *= a, O.w *= a;
#pragma unroll
                for (int j = 0; j < CB; ++j) {
                    const float w = c0 + j < nch ? expf(ml[j].x - mb) : 0.0f;
                    L += w * ml[j].y;
                    O.x += w * oc[j].x, O.y += w * oc[j].y, O.z += w * oc[j].z, O.w += w * oc[j].w;
                }
                M = mb;
            }
            *reinterpret_cast<float4 *>(s.xs + e) = make_float4(O.x / L, O.y / L, O.z / L, O.w / L);
        }
    }
    lds_barrier();
    quantize<NP>(s.xs, K, kquant, s.a);
}

// Ends the live range of a register group without code: the next phase's groups are loaded
// only by waves 1-7 (and the attention rows only by active workgroups), so without a
// definition on every path the previous values would stay live around the whole step loop.
__device__ __forceinline__ void kill(Frag &f) { asm volatile("" : "=v"(f.a), "=v"(f.b), "=v"(f.c), "=v"(f.e)); }
template <int N>
__device__ __forceinline__ void kill(Frag (&f)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) kill(f[i]);
}
template <int N>
__device__ __forceinline__ void kill(h8 (&r)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "=v"(r[i]));
}

template <bool KQ, class F>
__device__ __forceinline__ void with_t(int t, F &&f) {
    if constexpr (KQ) {
        if (t == 14)
            f.template operator()<14>();
        else
            f.template operator()<12>();
    } else {
        f.template operator()<8>();
    }
}

// wave 0: poll the 8 counter shards until they sum to `target` (false: timeout or another
// workgroup's error)
__device__ bool poll_shards(unsigned *ctl, unsigned target) {
    const int lane = MIO_TIDX & 63;
    for (int spins = 0;; ++spins) {
        unsigned v = 0, e = 0;
        if (lane < 8) v = __hip_atomic_load(ctl + lane * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 8) e = __hip_atomic_load(ctl + 256, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 1);
        const unsigned tot = __builtin_amdgcn_readfirstlane(v);
        const unsigned err = __builtin_amdgcn_readlane(e, 8);
        if (err) return false;
        if (tot >= target) return true;
        if (spins > kSpinLimit) {
            if (lane == 0) __hip_atomic_store(ctl + 256, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// Compile-time shape of one instantiation: passes for n_embd / n_ff, weight family, head
// dim, q heads per kv head, single-group sizes of the four layer matvecs (0 = streaming).
template <int NPE_, int NPF_, bool KQ_, int HD_, int GQ_, int SAI_, int SAO_, int SFI_, int SFD_>
struct PCfg {
    static constexpr int NPE = NPE_, NPF = NPF_, HD = HD_, GQ = GQ_;
    static constexpr bool KQ = KQ_;
    static constexpr int SAI = SAI_, SAO = SAO_, SFI = SFI_, SFD = SFD_;
};

// LDS carve (byte offsets, 16-aligned): flags | xcur[E] | xnw[E] | xin[XI] | smem(Kmax) |
// qs[GQ][HD] | knew[HD] | vnew[HD] | wres[8][GQ][HD+2]
struct PLds {
    size_t flags, xcur, xnw, xin, sm, qs, knew, vnew, wres, total;
};
__host__ __device__ inline size_t al16(size_t v) { return (v + 15) & ~(size_t)15; }
__host__ __device__ inline PLds plds(int E, int F, int HD, int GQ, int G) {
    PLds p;
    const int kmax = E > F ? E : F;
    int xi = F > E ? F : E;
    if (xi < (GQ + 2) * HD) xi = (GQ + 2) * HD;
    if (xi < 2 * G) xi = 2 * G;
    size_t o = 0;
    p.flags = o, o += 64;
    p.xcur = o, o = al16(o + (size_t)E * 4);
    p.xnw = o, o = al16(o + (size_t)E * 4);
    p.xin = o, o = al16(o + (size_t)xi * 4);
    p.sm = o, o = al16(o + smem_bytes(kmax));
    p.qs = o, o = al16(o + (size_t)GQ * HD * 4);
    p.knew = o, o = al16(o + (size_t)HD * 4);
    p.vnew = o, o = al16(o + (size_t)HD * 4);
    p.wres = o, o = al16(o + (size_t)MW * GQ * (HD + 2) * 4);
    p.total = o;
    return p;
}

// Read-only tables of the launch through the scalar path (constant address space): the
// layer table and the sampling config are written by the host before the launch, so every
// weight pointer stays in SGPRs (a generic-pointer load would land in VGPRs and turn every
// buffer load into a waterfall loop).
typedef const __attribute__((address_space(4))) LayerW CLayerW;
typedef const __attribute__((address_space(4))) SampleCfg CSampleCfg;

typedef const __attribute__((address_space(4))) QMat CQMat;
__device__ __forceinline__ QMat ldq(CQMat &q) {
    QMat r;
    r.type = q.type, r.rows = q.rows, r.k = q.k;
    r.p0 = q.p0, r.p1 = q.p1, r.p2 = q.p2, r.p3 = q.p3;
    return r;
}
// a layer's table entry by scalar loads (unused fields are never loaded)
__device__ __forceinline__ LayerW ldl(CLayerW &L) {
    LayerW r;
    r.attn_norm = L.attn_norm, r.q_norm = L.q_norm, r.k_norm = L.k_norm, r.ffn_norm = L.ffn_norm;
    r.wq = ldq(L.wq), r.wk = ldq(L.wk), r.wv = ldq(L.wv), r.wo = ldq(L.wo);
    r.gate = ldq(L.gate), r.up = ldq(L.up), r.down = ldq(L.down);
    return r;
}

template <class C>
__global__ __launch_bounds__(MT) void k_persist(PersistArgs A) {
    constexpr int NPE = C::NPE, NPF = C::NPF, HD = C::HD, GQ = C::GQ;
    constexpr bool KQ = C::KQ;
    using AC = AttCfg<HD>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const LlmDims &d = A.d;
    const LlmBuffers &b = A.b;
    const int G = gridDim.x, bid = blockIdx.x;
    const int lane = MIO_TIDX & 63, wave = __builtin_amdgcn_readfirstlane(MIO_TIDX >> 6);
    const int E = d.n_embd, F = d.n_ff;
    const PLds P = plds(E, F, HD, GQ, G);
    int *flags = (int *)(smem + P.flags);  // [0] abort, [1] sampled token
    float *xcur = (float *)(smem + P.xcur), *xnw = (float *)(smem + P.xnw), *xin = (float *)(smem + P.xin);
    const Smem s = carve(smem + P.sm, E > F ? E : F);
    float(*qs)[HD] = (float(*)[HD])(smem + P.qs);
    float *knew = (float *)(smem + P.knew), *vnew = (float *)(smem + P.vnew);
    float(*wres)[GQ][HD + 2] = (float(*)[GQ][HD + 2])(smem + P.wres);
    unsigned *ctl = A.ctl;
    // diagnostic phase timeline (mio_hip_llm_persist_timeline): per phase and workgroup
    // {0 body start, 1 prologue done, 2 body done, 3 arrived, 4 poll done, 5 staged,
    //  6 prefetch issued} in s_memrealtime ticks; thread 0 (wave 0) or 64 (wave 1) stamps
    int seq = 0;
    auto mark = [&](int k, unsigned t) {
        if (A.tl && MIO_TIDX == t) A.tl[((size_t)seq * G + bid) * 8 + k] = __builtin_amdgcn_s_memrealtime();
    };
    CLayerW *layers = (CLayerW *)A.layers;
    CSampleCfg &scc = *(CSampleCfg *)b.cfg;
    SampleCfg sc;
    sc.temp = scc.temp, sc.seed_lo = scc.seed_lo, sc.seed_hi = scc.seed_hi, sc.lo = scc.lo, sc.hi = scc.hi;
    sc.eos0 = scc.eos0, sc.eos1 = scc.eos1, sc.force = scc.force, sc.n_force = scc.n_force;
    sc.out_tokens = scc.out_tokens, sc.max_steps = scc.max_steps;
    const uint64_t seed = ((uint64_t)sc.seed_hi << 32) | sc.seed_lo;
    int pos = __builtin_amdgcn_readfirstlane(b.st->pos), step = __builtin_amdgcn_readfirstlane(b.st->step);
    unsigned ep = 0;
    if (MIO_TIDX == 0) flags[0] = 0;

    // ---- per-phase row ownership (layer independent)
    const int o1 = d.n_head * HD, o2 = o1 + d.n_kv * HD, rows_ai = o2 + d.n_kv * HD;
    int g_qk = (G * o2 + rows_ai / 2) / rows_ai;
    g_qk = g_qk < 1 ? 1 : (g_qk > G - 1 ? G - 1 : g_qk);
    const bool ai_qk = bid < g_qk;
    int ai_lo, ai_hi, ao_lo, ao_hi, fi_lo, fi_hi, fd_lo, fd_hi, lm_lo, lm_hi;
    if (ai_qk)
        wave_range_n(o2, ai_lo, ai_hi, bid, g_qk, 1, PW);
    else
        wave_range_n(d.n_kv * HD, ai_lo, ai_hi, bid - g_qk, G - g_qk, 1, PW);
    wave_range_n(E, ao_lo, ao_hi, bid, G, 1, PW);
    wave_range_n(F, fi_lo, fi_hi, bid, G, 1, PW);
    wave_range_n(E, fd_lo, fd_hi, bid, G, 1, PW);
    wave_range_n(d.n_vocab, lm_lo, lm_hi, bid, G, 1, PW);
    // attention item of this workgroup: (chunk, kv head), fixed for the whole launch, so a
    // chunk's K/V rows are always appended and read by the same workgroup
    const int at_ch = bid / d.n_kv, at_kvh = bid - (bid / d.n_kv) * d.n_kv;
    const bool at_slot = bid < d.max_splits * d.n_kv;
    const size_t layer_kv = (size_t)d.n_kv * d.n_ctx * HD;

    // ---- register groups (prefetched one phase ahead)
    Frag ai_a[Cfg<NPE, C::SAI>::U], ai_b[Cfg<NPE, C::SAI>::U];
    Frag ao_a[Cfg<NPE, C::SAO>::U], ao_b[Cfg<NPE, C::SAO>::U];
    Frag fi_a[Cfg<NPE, C::SFI>::U], fi_b[Cfg<NPE, C::SFI>::U];
    Frag fd_a[Cfg<NPF, C::SFD>::U], fd_b[Cfg<NPF, C::SFD>::U];
    Frag lm_a[Cfg<NPE>::U], lm_b[Cfg<NPE>::U];
    h8 kr[AC::IT], vr[AC::IT];

    auto pf_ai = [&](const LayerW &L) {
        if (ai_qk)
            with_t<KQ>(L.wq.type, [&]<int T>() { load_first<T, NPE, 1, C::SAI>(L.wq, L.wk, ai_lo, ai_hi, ai_a, ai_b, o1); });
        else
            with_t<KQ>(L.wv.type, [&]<int T>() { load_first<T, NPE, 1, C::SAI>(L.wv, L.wv, ai_lo, ai_hi, ai_a, ai_b); });
    };
    auto pf_ao = [&](const LayerW &L) {
        with_t<KQ>(L.wo.type, [&]<int T>() { load_first<T, NPE, 1, C::SAO>(L.wo, L.wo, ao_lo, ao_hi, ao_a, ao_b); });
    };
    auto pf_fi = [&](const LayerW &L) {
        with_t<KQ>(L.gate.type, [&]<int T>() { load_first<T, NPE, 2, C::SFI>(L.gate, L.up, fi_lo, fi_hi, fi_a, fi_b); });
    };
    auto pf_fd = [&](const LayerW &L) {
        with_t<KQ>(L.down.type, [&]<int T>() { load_first<T, NPF, 1, C::SFD>(L.down, L.down, fd_lo, fd_hi, fd_a, fd_b); });
    };
    auto pf_lm = [&]() {
        with_t<KQ>(A.lm.type, [&]<int T>() { load_first<T, NPE, 1>(A.lm, A.lm, lm_lo, lm_hi, lm_a, lm_b); });
    };
    auto at_active = [&]() { return at_slot && at_ch * ATT_CHUNK <= pos; };
    auto pf_kv = [&](int il) {  // the chunk's K/V rows (row `pos` itself comes from LDS)
        if (at_active())
            load_kv_rows<HD, true>(A.kc + il * layer_kv + (size_t)at_kvh * d.n_ctx * HD,
                             A.vc + il * layer_kv + (size_t)at_kvh * d.n_ctx * HD, at_ch * ATT_CHUNK, pos, kr, vr);
    };

    // ---- phase hand-off: drain, arrive, (waves 1-7) prefetch | (wave 0) poll + stage.
    // kl() ends the live range of the next phase's register groups on wave 0's path (which
    // never loads them), AFTER its staging, so the staging registers do not add to them.
    auto handoff = [&](auto &&pf, auto &&fetch, auto &&kl) -> bool {
        mark(2, 64);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        mark(3, 0);
        ++ep;
        if (wave == 0) {
            if (lane == 0)
                __hip_atomic_fetch_add(ctl + (bid & 7) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (poll_shards(ctl, ep * (unsigned)G)) {
                mark(4, 0);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                fetch();
                mark(5, 0);
            } else if (lane == 0) {
                flags[0] = 1;
            }
            kl();
        } else {
            pf();
            mark(6, 64);
        }
        lds_barrier();
        ++seq;
        mark(0, 0);
        return flags[0] == 0;
    };
    auto stage_x = [&](const float *nw) {  // residual stream x (sc1) + a norm weight
        stage<8, AUX_SC1>(xcur, b.x, E);
        stage<8, 0>(xnw, nw, E);
    };

    // ---- first phase of the launch: inputs from the previous launch (kernel boundary)
    if (wave == 0) {
        stage_x(layers[0].attn_norm);
        kill(ai_a), kill(ai_b);
    } else {
        pf_ai(ldl(layers[0]));
    }
    lds_barrier();
    mark(0, 0);

    for (int it = 0; it < A.n_steps; ++it) {
        for (int il = 0; il < d.n_layer; ++il) {
            const LayerW L = ldl(layers[il]);
            // ---------------- attn_in: RMSNorm -> quantize -> q|k|v rows (k_attn_in)
            {
                XRegs<NPE> xr;
                lds_xregs(xcur, xnw, E, xr);
                rmsnorm_quant(xr, E, d.eps, KQ, s);
                mark(1, 64);
                if (ai_qk)
                    with_t<KQ>(L.wq.type, [&]<int T>() {
                        stream_rows<T, NPE, 1, C::SAI>(L.wq, L.wk, ai_lo, ai_hi, ai_a, ai_b, s.a, [&](int row, float v, float) {
                            if (lane == 0) st_sc1(b.qkv + row, v);
                        }, o1);
                    });
                else
                    with_t<KQ>(L.wv.type, [&]<int T>() {
                        stream_rows<T, NPE, 1, C::SAI>(L.wv, L.wv, ai_lo, ai_hi, ai_a, ai_b, s.a, [&](int row, float v, float) {
                            if (lane == 0) st_sc1(b.qkv + o2 + row, v);
                        });
                    });
            }
            if (!handoff(
                    [&] {
                        kill(kr), kill(vr);
                        pf_kv(il);
                    },
                    [&] {
                        if (at_active()) {  // q heads of the kv head, k and v rows -> xin
                            stage<2, AUX_SC1>(xin, b.qkv + (size_t)at_kvh * GQ * HD, GQ * HD);
                            stage<1, AUX_SC1>(xin + GQ * HD, b.qkv + o1 + (size_t)at_kvh * HD, HD);
                            stage<1, AUX_SC1>(xin + (GQ + 1) * HD, b.qkv + o2 + (size_t)at_kvh * HD, HD);
                        }
                    },
                    [&] {
                        kill(kr), kill(vr);
                        pf_kv(il);
                    }))
                return;
            // ---------------- attention chunk (k_attention)
            if (at_active()) {
                constexpr int PER = HD / 64;
                const int t0 = at_ch * ATT_CHUNK;
                const float2 *rope = b.rope + (size_t)pos * (HD / 2);
                _Float16 *kc = A.kc + il * layer_kv, *vc = A.vc + il * layer_kv;
                const bool owner = pos < t0 + ATT_CHUNK;
                for (int hh = wave; hh < GQ + (owner ? 1 : 0); hh += ATT_NW) {
                    const bool isk = hh == GQ;
                    float vv[PER];
                    if (isk) {
#pragma unroll
                        for (int i = 0; i < PER; ++i) vv[i] = xin[(GQ + 1) * HD + lane + 64 * i];
                    }
                    const float *src = isk ? xin + GQ * HD : xin + hh * HD;
                    prep_head<HD>(src, isk ? L.k_norm : L.q_norm, rope, d, isk ? knew : qs[hh]);
                    if (isk) {
                        _Float16 *kd = kc + ((size_t)at_kvh * d.n_ctx + pos) * HD;
                        _Float16 *vd = vc + ((size_t)at_kvh * d.n_ctx + pos) * HD;
#pragma unroll
                        for (int i = 0; i < PER; ++i) {
                            const int p = lane + 64 * i;
                            const float vr16 = f16r(vv[i]);
                            vnew[p] = vr16;
                            kd[p] = (_Float16)knew[p];
                            vd[p] = (_Float16)vr16;
                        }
                    }
                }
                lds_barrier();
                mark(1, 64);
                if (owner) {
                    const int sl = MIO_TIDX / AC::LP, lp = lane % AC::LP, r = pos - t0;
                    if (sl == r % AC::NS) {
                        h8 kn, vn;
#pragma unroll
                        for (int i = 0; i < 8; ++i) kn[i] = (_Float16)knew[lp * 8 + i], vn[i] = (_Float16)vnew[lp * 8 + i];
#pragma unroll
                        for (int q = 0; q < AC::IT; ++q)
                            if (q == r / AC::NS) kr[q] = kn, vr[q] = vn;
                    }
                }
                attend_chunk<HD, GQ, true>(qs, kr, vr, t0, pos, d.scale, wres,
                                           b.part + ((size_t)(at_kvh * GQ) * d.max_splits + at_ch) * AC::REC,
                                           (size_t)d.max_splits * AC::REC);
            }
            if (!handoff([&] { pf_ao(L); }, [] {}, [&] { kill(ao_a), kill(ao_b); })) return;
            // ---------------- attn_out: chunk merge -> quantize -> O rows + residual (k_attn_out)
            {
                merge_attention_sc1<NPE>(d, b.part, pos / ATT_CHUNK + 1, E, KQ, s);
                mark(1, 64);
                with_t<KQ>(L.wo.type, [&]<int T>() {
                    stream_rows<T, NPE, 1, C::SAO>(L.wo, L.wo, ao_lo, ao_hi, ao_a, ao_b, s.a, [&](int row, float v, float) {
                        if (lane == 0) st_sc1(b.x + row, v + xcur[row]);
                    });
                });
            }
            if (!handoff([&] { pf_fi(L); }, [&] { stage_x(L.ffn_norm); }, [&] { kill(fi_a), kill(fi_b); })) return;
            // ---------------- ffn_in: RMSNorm -> quantize -> gate|up -> silu(g)*u (k_ffn_in)
            {
                XRegs<NPE> xr;
                lds_xregs(xcur, xnw, E, xr);
                rmsnorm_quant(xr, E, d.eps, KQ, s);
                mark(1, 64);
                with_t<KQ>(L.gate.type, [&]<int T>() {
                    stream_rows<T, NPE, 2, C::SFI>(L.gate, L.up, fi_lo, fi_hi, fi_a, fi_b, s.a, [&](int row, float g, float u) {
                        if (lane == 0) st_sc1(b.h + row, silu_f(g) * u);
                    });
                });
            }
            if (!handoff([&] { pf_fd(L); }, [&] { stage<24, AUX_SC1>(xin, b.h, F); }, [&] { kill(fd_a), kill(fd_b); }))
                return;
            // ---------------- ffn_down: quantize h -> down rows + residual (k_ffn_down)
            {
                XRegs<NPF> xr;
                lds_xregs(xin, nullptr, F, xr);
                plain_quant(xr, F, KQ, s);
                mark(1, 64);
                with_t<KQ>(L.down.type, [&]<int T>() {
                    stream_rows<T, NPF, 1, C::SFD>(L.down, L.down, fd_lo, fd_hi, fd_a, fd_b, s.a, [&](int row, float v, float) {
                        if (lane == 0) st_sc1(b.x + row, v + xcur[row]);
                    });
                });
            }
            const bool last = il + 1 == d.n_layer;
            if (!handoff(
                    [&] {
                        kill(ai_a), kill(ai_b), kill(lm_a), kill(lm_b);
                        if (last)
                            pf_lm();
                        else
                            pf_ai(ldl(layers[il + 1]));
                    },
                    [&] { stage_x(last ? A.out_norm : layers[il + 1].attn_norm); },
                    [&] { kill(ai_a), kill(ai_b), kill(lm_a), kill(lm_b); }))
                return;
        }
        // ---------------- lm_head + per-workgroup Gumbel-max (k_lm_head)
        {
            XRegs<NPE> xr;
            lds_xregs(xcur, xnw, E, xr);
            rmsnorm_quant(xr, E, d.eps, KQ, s);
            mark(1, 64);
            float r0 = -INFINITY, r1 = -INFINITY;
            with_t<KQ>(A.lm.type, [&]<int T>() {
                stream_rows<T, NPE, 1>(A.lm, A.lm, lm_lo, lm_hi, lm_a, lm_b, s.a, [&](int row, float v, float) {
                    const int k = row - lm_lo;
                    r0 = lane == k ? v : r0;
                    r1 = lane + 64 == k ? v : r1;
                });
            });
            float best = -INFINITY;
            int bi = INT_MAX;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int row = lm_lo + lane + 64 * h;
                const float v = h ? r1 : r0;
                if (row < lm_hi) {
                    b.logits[row] = v;
                    if (row >= sc.lo && row < sc.hi) {
                        const float t = sc.temp > 0.0f ? v / sc.temp + gumbel(seed, step, row) : v;
                        if (t > best || (t == best && row < bi)) best = t, bi = row;
                    }
                }
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                const float ov = __shfl_xor(best, o);
                const int oi = __shfl_xor(bi, o);
                if (ov > best || (ov == best && oi < bi)) best = ov, bi = oi;
            }
            float *wb = s.xs;  // free after the stream (the activation lives in s.a)
            int *wi = (int *)(s.xs + MW);
            if (lane == 0) wb[wave] = best, wi[wave] = bi;
            lds_barrier();
            if (MIO_TIDX == 0) {
                for (int w = 0; w < MW; ++w)
                    if (wb[w] > best || (wb[w] == best && wi[w] < bi)) best = wb[w], bi = wi[w];
                st_sc1(b.smp + 2 * bid, best);
                st_sc1(b.smp + 2 * bid + 1, __int_as_float(bi));
            }
        }
        const bool more = it + 1 < A.n_steps;
        if (!handoff(
                [&] {
                    kill(ai_a), kill(ai_b);
                    if (more) pf_ai(ldl(layers[0]));
                },
                [&] {  // every workgroup reduces the G partials (max value, then lowest id)
                    float best = -INFINITY;
                    int bi = INT_MAX;
                    for (int i = lane; i < G; i += 64) {
                        const auto r = __builtin_amdgcn_raw_buffer_load_b64(rsrc(b.smp, (uint32_t)G * 8), (uint32_t)i * 8, 0,
                                                                            AUX_SC1);
                        const float v = __uint_as_float(r[0]);
                        const int ix = (int)r[1];
                        if (v > best || (v == best && ix < bi)) best = v, bi = ix;
                    }
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) {
                        const float ov = __shfl_xor(best, o);
                        const int oi = __shfl_xor(bi, o);
                        if (ov > best || (ov == best && oi < bi)) best = ov, bi = oi;
                    }
                    if (lane == 0) flags[1] = bi;
                },
                [&] { kill(ai_a), kill(ai_b); }))
            return;
        // ---------------- sampler tail + next embedding (k_sample)
        {
            int tok = flags[1];
            if (tok == INT_MAX) tok = sc.lo;
            if (sc.force && step < sc.n_force && sc.force[step] >= 0) tok = sc.force[step];
            for (int e = MIO_TIDX; e < E; e += MT) xcur[e] = dequant_elem(A.tok, tok, e);
            if (more)
                for (int e = MIO_TIDX; e < E; e += MT) xnw[e] = layers[0].attn_norm[e];
            if (bid == 0 && MIO_TIDX == 0) {
                if (step < sc.max_steps) sc.out_tokens[step] = tok;
                if (tok == sc.eos0 || tok == sc.eos1) b.st->done = 1;
                b.st->token = tok;
                b.st->pos = pos + 1;
                b.st->step = step + 1;
            }
            ++pos;
            ++step;
            lds_barrier();
            if (!more && bid == 0)  // the residual stream for the next launch
                for (int e = MIO_TIDX; e < E; e += MT) b.x[e] = xcur[e];
        }
    }
}

// ------------------------------------------------------------------ instantiations
// (NPE, NPF, Q-family, head dim, q heads per kv head) of the synthetic presets, all with
// streaming groups; the 1.7B preset also with its single-group sizes at 256 CUs.
using PC_tiny_q8 = PCfg<1, 1, false, 64, 2, 0, 0, 0, 0>;
using PC_tiny_q4 = PCfg<1, 1, true, 64, 2, 0, 0, 0, 0>;
using PC_01b = PCfg<1, 1, false, 64, 3, 0, 0, 0, 0>;
using PC_26b = PCfg<1, 6, false, 64, 4, 0, 0, 0, 0>;
using PC_17b = PCfg<1, 3, true, 128, 2, 0, 0, 0, 0>;
using PC_17b_256 = PCfg<1, 3, true, 128, 2, 3, 2, 0, 0>;

// units (row passes) of the busiest row wave for `rows` rows over G workgroups
int units_of(int rows, int G, int np, int nm) {
    const int rg = (rows + G - 1) / G, rw = (rg + PW - 1) / PW;
    return rw * np * nm;
}

template <class C>
int go(const PersistArgs &a, int G, hipStream_t s) {
    const PLds P = plds(a.d.n_embd, a.d.n_ff, C::HD, C::GQ, G);
    const size_t lds = P.total < 82 * 1024 ? 82 * 1024 : P.total;  // > 80 KB: one workgroup per CU
    if (lds > 160 * 1024) return 1;
    static bool attr = false;  // per instantiation
    if (!attr) {
        if (hipFuncSetAttribute((const void *)k_persist<C>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
            hipSuccess)
            return 2;
        attr = true;
    }
    hipLaunchKernelGGL(k_persist<C>, dim3(G), dim3(MT), lds, s, a);
    return 0;
}
}  // namespace

size_t persist_ctl_bytes() { return 2048; }

int launch_persist(const PersistArgs &a, int G, hipStream_t s) {
    const LlmDims &d = a.d;
    if (G < 16 || G > 1024 || d.max_splits * d.n_kv > G || units_of(d.n_vocab, G, 1, 1) > 128 ||
        d.n_embd > 4 * MT * 6 || d.n_ff > 4 * MT * 6)
        return 1;
    const int npe = pick_np(d.n_embd), npf = pick_np(d.n_ff), GQ = d.n_head / d.n_kv;
    const bool kq = a.lm.type != 8;
    if (hipMemsetAsync(a.ctl, 0, persist_ctl_bytes(), s) != hipSuccess) return 2;
    if (npe == 1 && npf == 3 && kq && d.hd == 128 && GQ == 2) {
        const int rows_ai = (d.n_head + 2 * d.n_kv) * d.hd, o2 = (d.n_head + d.n_kv) * d.hd;
        int g_qk = (G * o2 + rows_ai / 2) / rows_ai;
        g_qk = g_qk < 1 ? 1 : (g_qk > G - 1 ? G - 1 : g_qk);
        const int uai = std::max(units_of(o2, g_qk, 1, 1), units_of(rows_ai - o2, G - g_qk, 1, 1));
        if (uai <= 3 && units_of(d.n_embd, G, 1, 1) <= 2) return go<PC_17b_256>(a, G, s);
        return go<PC_17b>(a, G, s);
    }
    if (npe == 1 && npf == 1 && !kq && d.hd == 64 && GQ == 2) return go<PC_tiny_q8>(a, G, s);
    if (npe == 1 && npf == 1 && kq && d.hd == 64 && GQ == 2) return go<PC_tiny_q4>(a, G, s);
    if (npe == 1 && npf == 1 && !kq && d.hd == 64 && GQ == 3) return go<PC_01b>(a, G, s);
    if (npe == 1 && npf == 6 && !kq && d.hd == 64 && GQ == 4) return go<PC_26b>(a, G, s);
    return 1;
}
}  // namespace mio
