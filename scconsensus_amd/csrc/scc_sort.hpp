// scc_sort.hpp — workgroup-wide bitonic sorting networks for CDNA4.
//
// The network is the "all ascending" bitonic form (each merge opens with a
// mirrored compare i <-> i ^ (size-1), then half-cleaners), so arrays of any
// length n sort in place: partners at index >= n are virtual +inf and are
// skipped, never moved.  Accessors hide SoA vs AoS and LDS vs HBM storage.
#pragma once
#include "scc_common.hpp"

// (orderable value key, cluster code) pairs, SoA: 9 B/element in LDS.
struct AccKeyCode {
    u64* k;
    u8* c;
    __device__ inline void cmpswap(int i, int j) const
    {
        u64 ki = k[i], kj = k[j];
        u8 ci = c[i], cj = c[j];
        if (kj < ki || (kj == ki && cj < ci)) {
            k[i] = kj;
            k[j] = ki;
            c[i] = cj;
            c[j] = ci;
        }
    }
    __device__ inline void put(int di, const AccKeyCode& src, int si) const
    {
        k[di] = src.k[si];
        c[di] = src.c[si];
    }
};

// generic records with operator<
template <class R>
struct AccAoS {
    R* r;
    __device__ inline void cmpswap(int i, int j) const
    {
        R a = r[i], b = r[j];
        if (b < a) {
            r[i] = b;
            r[j] = a;
        }
    }
    __device__ inline void put(int di, const AccAoS& src, int si) const { r[di] = src.r[si]; }
};

// one compare stage over [0, n): mirrored (rev) or half-cleaner with `stride`
template <class A>
__device__ inline void bitonic_stage(const A& a, int n, int m, int size, int stride, bool rev, int tid, int T)
{
    const int npairs = m >> 1;
    if (rev) {
        const int half = size >> 1;
        const int sh = __builtin_ctz(half);
        for (int q = tid; q < npairs; q += T) {
            const int i = ((q >> sh) << (sh + 1)) + (q & (half - 1));
            const int j = i ^ (size - 1);
            if (j < n) a.cmpswap(i, j);
        }
    } else {
        const int sh = __builtin_ctz(stride);
        for (int q = tid; q < npairs; q += T) {
            const int i = ((q >> sh) << (sh + 1)) + (q & (stride - 1));
            const int j = i + stride;
            if (j < n) a.cmpswap(i, j);
        }
    }
}

// Full sort of n elements living in one address space (LDS normally).
// A stage whose compare span (mirrored: size; half-cleaner: 2 stride) is at
// most 128 keeps every pair of wave w (pairs q in [64 w + T k, +64)) inside
// elements [128 (w + T/64 k), +128): between two such stages the wave's own
// order suffices (a wave barrier), and only the stages that span more than 128
// elements take a workgroup barrier (1024 elements: 10 of 55).
__device__ inline void bitonic_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <class A>
__device__ void block_bitonic(const A& a, int n, int tid, int T)
{
    if (n < 2) return;
    const int m = scc_next_pow2(n);
    auto sync = [&](int span, int next_span) {
        if (span <= 128 && next_span <= 128 && (T & 63) == 0)
            bitonic_wave_sync();
        else
            __syncthreads();
    };
    for (int size = 2; size <= m; size <<= 1) {
        bitonic_stage(a, n, m, size, 0, true, tid, T);
        // the next stage's span: the first half-cleaner's (2 * size / 4), else
        // the next merge's mirrored stage, else none (the end: a full barrier)
        const int nxt = (size >= 4) ? (size >> 1) : ((size << 1) <= m ? (size << 1) : (1 << 30));
        sync(size, nxt);
        for (int stride = size >> 2; stride > 0; stride >>= 1) {
            bitonic_stage(a, n, m, size, stride, false, tid, T);
            const int next = (stride > 1) ? stride : ((size << 1) <= m ? (size << 1) : (1 << 30));
            sync(2 * stride, next);
        }
    }
}

// Sort n elements in HBM (accessor g) using an LDS staging accessor s of CH
// elements (CH a power of two): chunks are sorted and finished in LDS; only
// the strides >= CH run against HBM (L2-resident for one gene / one pair).
template <class A>
__device__ void block_bitonic_staged(const A& g, int n, const A& s, int CH, int tid, int T)
{
    auto load = [&](int c0, int cn) {
        for (int i = tid; i < cn; i += T) s.put(i, g, c0 + i);
    };
    auto store = [&](int c0, int cn) {
        for (int i = tid; i < cn; i += T) g.put(c0 + i, s, i);
    };
    if (n <= CH) {
        load(0, n);
        __syncthreads();
        block_bitonic(s, n, tid, T);
        store(0, n);
        __syncthreads();
        return;
    }
    for (int c0 = 0; c0 < n; c0 += CH) {
        const int cn = min(CH, n - c0);
        load(c0, cn);
        __syncthreads();
        block_bitonic(s, cn, tid, T);
        store(c0, cn);
        __syncthreads();
    }
    const int m = scc_next_pow2(n);
    for (int size = 2 * CH; size <= m; size <<= 1) {
        bitonic_stage(g, n, m, size, 0, true, tid, T);
        __syncthreads();
        for (int stride = size >> 2; stride >= CH; stride >>= 1) {
            bitonic_stage(g, n, m, size, stride, false, tid, T);
            __syncthreads();
        }
        for (int c0 = 0; c0 < n; c0 += CH) {
            const int cn = min(CH, n - c0);
            load(c0, cn);
            __syncthreads();
            const int cm = scc_next_pow2(cn);
            for (int stride = CH >> 1; stride > 0; stride >>= 1) {
                if (stride < cm) bitonic_stage(s, cn, cm, 0, stride, false, tid, T);
                __syncthreads();
            }
            store(c0, cn);
            __syncthreads();
        }
    }
}
