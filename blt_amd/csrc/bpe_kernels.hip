// MI355X (gfx950, CDNA4) kernels for the BPE merge scan of jtrefon/blt.
//
// The reference (blt_core/src/tokenizer.rs:56-93) runs, per chunk, greedy left-to-right
// passes: at position i, if (t[i], t[i+1]) is in the merge map it emits the mapped token and
// skips 2, otherwise it emits t[i] and skips 1; passes repeat until one merges nothing; tokens
// are serialised big-endian u16.  Chunks are fixed-size slices of the input and never merge
// across a boundary (pipeline.rs:73-81), outputs are concatenated in chunk order
// (pipeline.rs:153-192).
//
// One pass is a scan.  Let m[i] = "(t[i], t[i+1]) is a merge and i is not the last position of
// its chunk", and L[i] = "the scan pointer lands on i".  Then L[0] = 1 and
// L[i+1] = !(L[i] && m[i]): a chunk start lands automatically because m is 0 at the position
// before it.  Position i emits iff L[i], emitting map[t[i], t[i+1]] when m[i] and t[i] otherwise;
// its output index is the number of landings before it.  Merges sit at even offsets of every
// run of 1s in m that starts on a landing, so a lane turns its 16-position mask into merge and
// landing masks with three integer ops (merges_for).  A segment's carry function is identity
// when all 16 positions merge and a constant otherwise, so carries resolve across a wave with
// two ballots and across the tile with the same trick on the per-wave summaries.
//
// Whole-buffer structure: one launch covers every chunk of the buffer.  The buffer is cut into
// super-tiles of kTilePos positions; a workgroup takes tiles from an atomic ticket (dynamic, so
// no residency assumption is needed for progress), computes the tile's carry/count function,
// publishes it, then resolves its carry-in and output offset by a decoupled look-back over
// 64-bit status words (Merrill & Garland single-pass scan) and writes its compacted tokens,
// staged through LDS, with 16-byte coalesced stores.  HBM traffic is one read of the input and
// one write of the output.
//
// Byte pass (every map loaded from a merges file, and pass 1 of every other map; seg::
// scan_bytes_kernel): the self-token table (entry (a, b) = the merged token, or a itself) lives in
// LDS as 256 rows of 258 u16 entries (129 KiB of the CU's 160 KiB); the 2-entry row pad skews rows
// across the banks and the entry address is one v_dot2_u32_u16 of the byte pair.  General u16
// maps (chained merges, byte-valued merges, u16 wrap) run extra passes on big-endian u16 tokens
// (seg::scan_tokens_kernel) with a bucket table of the map: one-probe (up to 512 keys) or
// 2-choice cuckoo buckets, in LDS up to 48 KiB, else read through L2.  merge_pass_kernel /
// merge_tokens_kernel below are the barrier-phased generic passes for what those two cannot take
// (byte maps with a merge whose value is its own first byte, chunks under 4 KiB, u16 passes over
// chunks under 1024 tokens).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stddef.h>

#include <atomic>
#include <mutex>
#include <unordered_map>

#include "bpe_kernels.h"

namespace blt {

constexpr int kThreads = 512;                 // generic passes: 8 waves per workgroup; the byte
                                              // table (128 KiB) allows one per CU, the u16 bucket
                                              // table (<= 48 KiB) several
constexpr int kWaves = kThreads / 64;
constexpr int kSeg = 16;                      // positions per lane per sub-tile
constexpr int kSubPos = kThreads * kSeg;      // 8192 positions per sub-tile
constexpr int kStageBytes = 2 * kSubPos + 32;
// Spin timeouts are wall-clock time (s_memrealtime, a constant 100 MHz clock), not iteration counts:
// a predecessor slowed by other work on the device (a co-tenant kernel, another queue's time slice)
// still finishes well inside them, so only a stuck wait is flagged (a count of
// sleeps is as long as the clock the waves happen to run at, milliseconds at best).
constexpr uint32_t kSpinTimeoutTicks = 20000000u;   // 200 ms at 100 MHz
// The clock is read once per kSpinClockEvery waits: s_memrealtime is a scalar-memory read, and
// waiting for it (lgkmcnt, the counter LDS reads share) on every spin made each wait's polling
// coarser: measured, the byte pass 8 % slower on cfg3 with a read per spin.
constexpr uint32_t kSpinClockEvery = 64;
struct SpinClock {
    uint32_t t0 = 0;   // low half of the clock (wraps every 43 s; the deltas here are far shorter)
    uint32_t n = 0;
    // true once the wait has lasted longer than kSpinTimeoutTicks (the first check starts the clock)
    __device__ __forceinline__ bool expired() {
        if ((++n % kSpinClockEvery) != 0u) return false;
        const uint32_t t = (uint32_t)__builtin_amdgcn_s_memrealtime();
        if (t0 == 0) { t0 = t | 1u; return false; }
        return t - t0 > kSpinTimeoutTicks;
    }
};
static_assert(kTilePos == kSub * kSubPos, "tile geometry");

__device__ __forceinline__ uint32_t swz_index(uint32_t a, uint32_t b) {
    return (a << 8) | (b ^ ((a << 1) & 0xFEu));   // = dense_index (bpe_kernels.h)
}

// Merge positions of a 16-position segment whose first position lands iff c.
__device__ __forceinline__ uint32_t merges_for(uint32_t m, uint32_t c) {
    uint32_t mc = c ? m : (m & ~1u);           // c = 0: position 0 was consumed by the previous merge
    uint32_t s = mc & ~(mc << 1);              // run starts
    uint32_t rodd = mc & ~(mc + (s & 0xAAAAu)); // runs that start at an odd position
    return (mc & ~rodd & 0x5555u) | (rodd & 0xAAAAu);
}

__device__ __forceinline__ uint32_t lands_for(uint32_t merges, uint32_t c, uint32_t valid) {
    return ~((merges << 1) | (c ^ 1u)) & valid & 0xFFFFu;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// Given per-lane {identity?, const carry-out} and counts under carry-in 0/1, resolves each
// lane's carry-in under both hypotheses for the first lane's carry-in.  Returns the packed
// (cnt|carry-in=0) | (cnt|carry-in=1) << 16 inclusive prefix; fills lane carry info and the
// wave's function.
struct WaveFn {
    uint32_t ident, cout;   // identity function, or constant carry-out
    uint32_t cnt0, cnt1;    // total count for carry-in 0 / 1
};

__device__ __forceinline__ void resolve_wave(uint32_t ident, uint32_t cout, uint32_t cnt0, uint32_t cnt1,
                                             int lane, uint32_t& has_below, uint32_t& below_cout,
                                             uint32_t& excl, WaveFn& fn) {
    uint64_t nonid = __ballot(!ident);
    uint64_t cmask = __ballot(cout);
    uint64_t below = nonid & ((1ull << lane) - 1ull);
    has_below = below != 0;
    below_cout = has_below ? (uint32_t)((cmask >> (63 - __clzll(below))) & 1ull) : 0u;
    uint32_t c0 = has_below ? below_cout : 0u;
    uint32_t c1 = has_below ? below_cout : 1u;
    uint32_t packed = (c0 ? cnt1 : cnt0) | ((c1 ? cnt1 : cnt0) << 16);
    uint32_t incl = wave_incl_scan(packed, lane);
    excl = incl - packed;
    uint32_t tot = __shfl(incl, 63, 64);
    fn.ident = nonid == 0;
    fn.cout = nonid ? (uint32_t)((cmask >> (63 - __clzll(nonid))) & 1ull) : 0u;
    fn.cnt0 = tot & 0xFFFFu;
    fn.cnt1 = tot >> 16;
}

// ---- status words of the decoupled look-back (one per tile) -------------------------------
// bits 63..62: 0 empty, 1 aggregate, 2 inclusive prefix.
//  aggregate: bit 61 carry-out for carry-in 1, bit 60 for carry-in 0, bit 59 live (u16 scan
//             kernel: the tile has a merge whose value is a key component), bits 30..58 count
//             for carry-in 1, bits 0..29 count for carry-in 0.
//  inclusive: bit 61 carry into the next tile, bit 60 live (some tile up to this one is live),
//             bits 0..59 tokens before the next tile.
constexpr uint64_t kStLiveAgg = 1ull << 59, kStLiveIncl = 1ull << 60;
__device__ __forceinline__ uint64_t st_agg(uint32_t co0, uint32_t co1, uint32_t c0, uint32_t c1) {
    return (1ull << 62) | ((uint64_t)co1 << 61) | ((uint64_t)co0 << 60) | ((uint64_t)c1 << 30) | c0;
}
__device__ __forceinline__ uint64_t st_incl(uint32_t carry, uint64_t off) {
    return (2ull << 62) | ((uint64_t)carry << 61) | off;
}
__device__ __forceinline__ void st_publish(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t st_read(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Error bits into ctl[1] and the handle's sticky host word (vector stores only).
__device__ __forceinline__ void flag_error(uint32_t* ctl, uint32_t* sticky, uint32_t bit) {
    if (ctl) atomicOr(ctl + 1, bit);
    if (sticky) __hip_atomic_store(sticky, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A PassParams field read again from the kernel-argument segment where it is used (one scalar
// load; every kernel here takes the PassParams as its only argument), for fields the error,
// last-tile and record paths need: kept live across the persistent loops they would cost SGPRs the
// byte pass spills to VGPR lanes (34 spills, ~240 v_readlane in its body before this).
template <typename T>
__device__ __forceinline__ T karg_reload(size_t off) {
    typedef const volatile T __attribute__((address_space(4))) cvT;
    return *(cvT*)((const char __attribute__((address_space(4)))*)__builtin_amdgcn_kernarg_segment_ptr() + off);
}
#define KARG(field) karg_reload<decltype(PassParams::field)>(offsetof(PassParams, field))
// Per-tile debug records (tests/debug_replay.py, the timing tools) only in builds that ask for them.
#ifndef BLT_DEBUG_RECORD
#define BLT_DEBUG_RECORD 0
#endif
#ifdef BLT_TIMING
constexpr bool kDebugRecord = true;
#else
constexpr bool kDebugRecord = BLT_DEBUG_RECORD != 0;
#endif

// First failure wins: ctl[2] = T + 1, ctl[3] = sub-tile, ctl[4..5] = O, ctl[6..7] = value, ctl[8] = C.
__device__ void record_error(const PassParams& p, uint32_t bit, uint32_t T, uint32_t j, uint64_t O, uint64_t v,
                             uint32_t C) {
    flag_error(p.ctl, KARG(sticky), bit);
    if (atomicCAS(p.ctl + 2, 0u, T + 1u) == 0u) {
        p.ctl[3] = j;
        p.ctl[4] = (uint32_t)O; p.ctl[5] = (uint32_t)(O >> 32);
        p.ctl[6] = (uint32_t)v; p.ctl[7] = (uint32_t)(v >> 32);
        p.ctl[8] = C;
    }
}

// Self-reset of a single-pass launch: the last workgroup to leave zeroes the ticket and the
// status words (every look-back is over by then), so the next launch on this workspace needs no
// memset (BLT_ENCODE_WORKSPACE_ZEROED).  The error flags and first-error record stay.  Each
// wave's stores are acknowledged (vmcnt(0): the status publishes are agent-scope atomics, acked at
// the coherence point) before its workgroup counts itself out, so a late publish cannot land after
// the zeroing; the zeroing itself reaches the next launch through the kernel-end writeback.  (An
// agent-scope fence here writes back and invalidates the XCD's L2 under the workgroups still
// running: measured, the kernel 75 us slower.)  flag: a workgroup-shared word the caller is done with.
__device__ __forceinline__ void self_reset(const PassParams& p, uint32_t ntiles, uint32_t* flag) {
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    __syncthreads();
    if (threadIdx.x == 0)
        *flag = __hip_atomic_fetch_add(p.ctl + kCtlLeft, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u;
    __syncthreads();
    if (*flag) {
        uint4* st = reinterpret_cast<uint4*>(p.status);   // 16-byte aligned (after the control block)
        const uint32_t units = (ntiles + 1u) / 2u;         // within the zeroed region (rounded to 16 bytes)
        for (uint32_t i = threadIdx.x; i < units; i += blockDim.x) st[i] = make_uint4(0u, 0u, 0u, 0u);
        if (threadIdx.x == 0) {
            p.ctl[0] = 0u;
            p.ctl[kCtlLeft] = 0u;
            // words [0, ntiles) are zero now, and the ones past them were before (untouched here)
            if (ntiles > p.ctl[kCtlCover]) p.ctl[kCtlCover] = ntiles;
        }
    }
}

// A launch told its workspace is zeroed (p.ws_check) whose tiles reach past the status words known
// zero refuses: error bit 32 (one workgroup flags it) and no output; its workgroups claim no tile
// but still count themselves out, so the self-reset zeroes its ntiles words as usual.  The word is
// read at the workgroup's start (written before the launch on its stream) and tested after the
// table copy, off the critical path.  A relaxed atomic load, not a volatile one: measured, the
// volatile load (which the backend orders with waits) made the headline byte pass 6 % slower
// (cfg3 0.556 -> 0.590 ms, the check compiled out 0.554).
__device__ __forceinline__ uint32_t ws_cover(const PassParams& p) {
    return p.ws_check ? __hip_atomic_load(p.ctl + kCtlCover, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0xFFFFFFFFu;
}
__device__ __forceinline__ bool ws_refused(const PassParams& p, uint32_t ntiles, uint32_t cover) {
    if (ntiles <= cover) return false;
    if (blockIdx.x == 0 && threadIdx.x == 0) flag_error(p.ctl, KARG(sticky), 32u);
    return true;
}

// 16 x the lane index, computed where it is used: inline asm is never hoisted, so a rare branch
// (a chunk or buffer end in a wave range) does not keep a per-lane constant live across the
// byte pass's loop (the register allocator spilled two such VGPRs to scratch).
__device__ __forceinline__ uint32_t lane16_here() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0\n\tv_lshlrev_b32 %0, 4, %0" : "=v"(l));
    return l;
}

// Lane i's 64-bit value from its two halves.  readlane returns int: cast each half to uint32_t
// before widening, or the low half sign-extends over the flag and carry bits.
__device__ __forceinline__ uint64_t readlane_u64(uint32_t lo, uint32_t hi, int i) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, i) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, i);
}

struct Fn64 {  // tile-sequence function: carry-in c -> (carry-out, count)
    uint32_t co0, co1;
    uint64_t c0, c1;
};

// Wave-wide look-back for tile T (all 64 lanes of one wave).  Returns carry-in and the number
// of tokens before tile T.
__device__ void lookback(const PassParams& p, uint32_t T, uint32_t& C, uint64_t& O, uint32_t& how,
                         uint32_t* spins_out = nullptr) {
    const int lane = threadIdx.x & 63;
    Fn64 acc = {0u, 1u, 0ull, 0ull};   // function of tiles (k+1 .. T-1), identity so far
    int64_t k = (int64_t)T - 1;
    uint32_t spins = 0;
    SpinClock clk;
    for (;;) {
        int64_t idx = k - lane;
        uint64_t s = idx < 0 ? st_incl(1u, 0ull) : st_read(p.status + idx);
        uint32_t flag = (uint32_t)(s >> 62);
        uint64_t incl = __ballot(flag == 2u);
        uint64_t ready = __ballot(flag != 0u);
        int f = incl ? (int)__ffsll((unsigned long long)incl) - 1 : 64;
        uint64_t need = f >= 63 ? ~0ull : ((2ull << f) - 1ull);
        if ((ready & need) != need) {
            ++spins;
            if (clk.expired()) {   // flagged; the tile writes nothing (C = 2)
                if (lane == 0) flag_error(p.ctl, KARG(sticky), 1u);
                C = 2u; O = 0ull;
                return;
            }
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        uint32_t lo = (uint32_t)s, hi = (uint32_t)(s >> 32);
        if (f < 64) {
            uint64_t sf = readlane_u64(lo, hi, f);
            uint32_t carry = (uint32_t)(sf >> 61) & 1u;
            uint64_t off = sf & ((1ull << 61) - 1ull);
            for (int i = f - 1; i >= 0; --i) {
                uint64_t si = readlane_u64(lo, hi, i);
                off += carry ? ((si >> 30) & 0x3FFFFFFFull) : (si & 0x3FFFFFFFull);
                carry = carry ? (uint32_t)(si >> 61) & 1u : (uint32_t)(si >> 60) & 1u;
            }
            off += carry ? acc.c1 : acc.c0;
            carry = carry ? acc.co1 : acc.co0;
            C = carry; O = off;
            how = (uint32_t)f | ((uint32_t)(T - 1 - k) << 8);
            if (spins_out) *spins_out = spins;
            return;
        }
        // no inclusive prefix in the window: fold the 64 aggregates (tiles k-63 .. k) in front of acc
        Fn64 w = {0u, 1u, 0ull, 0ull};
        for (int i = 63; i >= 0; --i) {
            uint64_t si = readlane_u64(lo, hi, i);
            uint32_t aco0 = (uint32_t)(si >> 60) & 1u, aco1 = (uint32_t)(si >> 61) & 1u;
            uint64_t ac0 = si & 0x3FFFFFFFull, ac1 = (si >> 30) & 0x3FFFFFFFull;
            Fn64 nw;
            nw.c0 = w.c0 + (w.co0 ? ac1 : ac0);
            nw.c1 = w.c1 + (w.co1 ? ac1 : ac0);
            nw.co0 = w.co0 ? aco1 : aco0;
            nw.co1 = w.co1 ? aco1 : aco0;
            w = nw;
        }
        Fn64 na;
        na.c0 = w.c0 + (w.co0 ? acc.c1 : acc.c0);
        na.c1 = w.c1 + (w.co1 ? acc.c1 : acc.c0);
        na.co0 = w.co0 ? acc.co1 : acc.co0;
        na.co1 = w.co1 ? acc.co1 : acc.co0;
        acc = na;
        k -= 64;
    }
}

// ---- chunk boundaries ------------------------------------------------------------------
// First chunk start >= x (x < n), with its chunk index; returns pos >= n when none.
__device__ __forceinline__ uint64_t first_boundary(const PassParams& p, uint64_t x, uint64_t& kidx) {
    if (p.cs) {
        uint64_t k = (x + p.cs - 1) / p.cs;
        kidx = k;
        uint64_t pos = k * p.cs;
        return pos < p.n ? pos : p.n;
    }
    uint64_t lo = 0, hi = p.nchunks;  // lower_bound over cstart[0 .. nchunks)
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if (p.cstart[mid] < x) lo = mid + 1; else hi = mid;
    }
    kidx = lo;
    return lo < p.nchunks ? p.cstart[lo] : p.n;
}
__device__ __forceinline__ uint64_t next_boundary(const PassParams& p, uint64_t kidx) {
    if (p.cs) { uint64_t pos = (kidx + 1) * p.cs; return pos < p.n ? pos : p.n; }
    return kidx + 1 < p.nchunks ? p.cstart[kidx + 1] : p.n;
}

// ---- position loads ---------------------------------------------------------------------
template <typename InT> struct Seg;

template <> struct Seg<uint8_t> {
    uint32_t w[4];
    __device__ __forceinline__ void load(const uint8_t* in, uint64_t pos, uint64_t n) {
        if (pos + 16 <= n) {
            uint4 v = *reinterpret_cast<const uint4*>(in + pos);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) w[i] = 0;
            for (int k = 0; k < 16; ++k)
                if (pos + k < n) w[k >> 2] |= (uint32_t)in[pos + k] << (8 * (k & 3));
        }
    }
    __device__ __forceinline__ uint32_t at(int k) const { return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu; }
    static __device__ __forceinline__ uint32_t load1(const uint8_t* in, uint64_t pos) { return in[pos]; }
};

template <> struct Seg<uint16_t> {
    uint32_t w[8];
    __device__ __forceinline__ void load(const uint16_t* in, uint64_t pos, uint64_t n) {
        if (pos + 16 <= n) {
            uint4 a = *reinterpret_cast<const uint4*>(in + pos);
            uint4 b = *reinterpret_cast<const uint4*>(in + pos + 8);
            w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
            w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = 0;
            for (int k = 0; k < 16; ++k)
                if (pos + k < n) w[k >> 1] |= (uint32_t)in[pos + k] << (16 * (k & 1));
        }
    }
    __device__ __forceinline__ uint32_t at(int k) const { return (w[k >> 1] >> (16 * (k & 1))) & 0xFFFFu; }
    static __device__ __forceinline__ uint32_t load1(const uint16_t* in, uint64_t pos) { return in[pos]; }
};

// Global -> LDS copy of n 16-byte units by nthr threads, kBatch loads in flight per thread
// before their stores (a rolled loop waits for every load: one L2/MALL round trip each).
template <int kBatch, typename T>
__device__ __forceinline__ void copy_to_lds(T* dst, const T* src, uint32_t n, uint32_t tid, uint32_t nthr) {
    for (uint32_t i0 = tid; i0 < n; i0 += kBatch * nthr) {
        T v[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k)   // unconditional (a clamped duplicate): no branch to wait at
            v[k] = src[i0 + k * nthr < n ? i0 + k * nthr : n - 1];
#pragma unroll
        for (int k = 0; k < kBatch; ++k)
            if (i0 + k * nthr < n) dst[i0 + k * nthr] = v[k];
    }
}

// General-map lookup of the pair key BE(a) | BE(b) << 16 (the two u16 words as stored): both
// candidate buckets are read (no probe loop); returns the matching bucket's value word,
// BE(v) | 1 << 31, or 0.  The bucket is the top bits of v_dot2_u32_u16(key, hmul).
typedef unsigned short hu16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t bucket_hash(uint32_t key, uint32_t mul, uint32_t shift) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(hu16x2, key), __builtin_bit_cast(hu16x2, mul), 0u, false) >> shift;
}
template <typename TabPtr>
__device__ __forceinline__ uint32_t bucket_get(const PassParams& p, TabPtr tab, uint32_t key) {
    const uint2 x = tab[bucket_hash(key, p.hmul1, p.hshift)];
    const uint2 y = tab[bucket_hash(key, p.hmul2, p.hshift)];
    return (x.x == key ? x.y : 0u) | (y.x == key ? y.y : 0u);
}

__device__ __forceinline__ uint32_t bswap16(uint32_t t) { return ((t & 0xFFu) << 8) | ((t >> 8) & 0xFFu); }

// One merge pass over the whole buffer.  InT = uint8_t: byte input, dense LDS table (maps the
// byte pass cannot take).  InT = uint16_t: big-endian token input (the previous pass's output),
// the bucket table in LDS (kHashLds, dynamic shared memory) or global memory; the token count
// comes from the device (p.n_dev) and a pass after one that merged nothing returns at once, so
// the host enqueues passes without waiting for their counts.  kBE: write big-endian u16, else
// native u16.
template <typename InT, bool kBE, bool kHashLds>
__device__ __forceinline__ void merge_pass_body(const PassParams& pin) {
    constexpr bool kDense = sizeof(InT) == 1;
    constexpr int kSubT = kSub;
    constexpr uint64_t kTileT = (uint64_t)kSubT * kSubPos;
    constexpr int kGroupsT = kSubT * kWaves;
    __shared__ __attribute__((aligned(16))) uint16_t s_tab[kDense ? 65536 : 8];
    extern __shared__ uint2 s_hash[];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[kStageBytes];
    __shared__ WaveFn s_wfn[kGroupsT];
    __shared__ uint32_t s_gin[kGroupsT][4];   // carry-in (H=0, H=1), offset (H=0, H=1)
    __shared__ uint32_t s_tfn[4];            // tile function: co0, co1, cnt0, cnt1
    __shared__ uint32_t s_ticket;
    __shared__ uint32_t s_C;
    __shared__ uint64_t s_O;
    // u16 passes: the tile's chunk starts (token positions from p.cstart), relative to the tile's
    // first position, 0xFFFF past the last; fetched in one parallel round per tile
    __shared__ uint16_t s_bnd[kDense ? 1 : kThreads];
    // a start on the next tile's first position is stored as kTileT itself: it must stay below the
    // 0xFFFF end marker (a 64K-position tile would wrap it to 0, a start at the tile's first position)
    static_assert(kTileT < 0xFFFFu, "s_bnd: tile-relative u16 chunk starts");

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    PassParams p = pin;
    if constexpr (!kDense) {
        if (p.done && __hip_atomic_load(p.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
        if (p.n_dev) {
            p.n = __hip_atomic_load(const_cast<uint64_t*>(p.n_dev), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            p.ntiles = (uint32_t)((p.n + kTileT - 1) / kTileT);
        }
        // the grid was sized for the input's bound; workgroups past the tiles there are leave
        // before copying the table (the ones below claim every ticket)
        if (blockIdx.x >= p.ntiles) return;
        // chained u16 passes (round 6, as the scan kernel): the next pass's status words and ticket
        // (the other set) zeroed here, with agent-scope stores beside this pass's ticket atomics
        if (p.status_zero) {
            const uint64_t live = gridDim.x < p.ntiles ? gridDim.x : p.ntiles;
            for (uint64_t i = (uint64_t)blockIdx.x * kThreads + tid; i < p.ntiles; i += live * kThreads)
                __hip_atomic_store(p.status_zero + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (blockIdx.x == 0 && tid == 0)
                __hip_atomic_store(p.ctl + (p.tick ^ kCtlTickAlt), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    const uint32_t cover = kDense ? ws_cover(p) : 0xFFFFFFFFu;
    const InT* in = reinterpret_cast<const InT*>(p.in);
    uint8_t* out = reinterpret_cast<uint8_t*>(p.out);

    if constexpr (kDense) {
        const uint4* src = reinterpret_cast<const uint4*>(p.dense);
        uint4* dst = reinterpret_cast<uint4*>(s_tab);
        copy_to_lds<8>(dst, src, 65536u * 2u / 16u, (uint32_t)tid, (uint32_t)kThreads);
    } else if constexpr (kHashLds) {
        copy_to_lds<8>(s_hash, p.hbuckets, p.hbytes / 8u, (uint32_t)tid, (uint32_t)kThreads);
    }

    const bool refused = kDense && ws_refused(p, p.ntiles, cover);
    for (;;) {
        if (refused) break;
        if (tid == 0) s_ticket = atomicAdd(p.ctl + p.tick, 1u);
        __syncthreads();
        const uint32_t T = s_ticket;
        if (T >= p.ntiles) break;
        const uint64_t tile0 = (uint64_t)T * kTileT;
        // Chunk starts of a u16 pass (p.cs == 0: p.cstart holds them, token positions): the
        // tile's first kThreads of them go to LDS in one round of parallel loads, and each lane
        // searches that list for its own 16 positions, instead of walking p.cstart one dependent
        // global load per chunk start, per sub-tile and twice per tile (measured on the f2 chain
        // row's tail passes, 16 chunks of a few hundred tokens: 22.6 -> 17.6 us per launch, the
        // row 0.86 -> 0.83 ms).  nb = kThreads: the list may be incomplete, and the tile walks
        // p.cstart as before.
        uint32_t nb = kThreads;
        uint64_t bk0 = 0;
        if constexpr (!kDense) {
            if (p.cs == 0) {
                (void)first_boundary(p, tile0, bk0);   // uniform: the same loads on every lane
                const uint64_t k = bk0 + (uint64_t)tid;
                uint32_t rel = 0xFFFFu;
                if (k < p.nchunks) {
                    const uint64_t b = p.cstart[k];
                    if (b < p.n && b <= tile0 + kTileT) rel = (uint32_t)(b - tile0);   // <= 32768
                }
                s_bnd[tid] = (uint16_t)rel;
                nb = (uint32_t)__syncthreads_count(rel != 0xFFFFu);   // chunk starts are increasing
            }
        }
        // first entry of s_bnd[0 .. nb) that is >= lo
        auto bnd_lower = [&](uint32_t lo) {
            uint32_t a = 0, z = nb;
            while (a < z) {
                const uint32_t mid = (a + z) >> 1;
                if (s_bnd[mid] < lo) a = mid + 1; else z = mid;
            }
            return a;
        };

        Seg<InT> seg[kSubT];
        uint32_t vals[kSubT][8];
        uint32_t mm[kSubT], valid[kSubT], hasb[kSubT], bco[kSubT], excl[kSubT];

        // ---- phase 1: lookups and per-lane / per-wave carry functions --------------------
#pragma unroll
        for (int j = 0; j < kSubT; ++j) {
            const uint64_t sub0 = tile0 + (uint64_t)j * kSubPos;
            const uint64_t pos = sub0 + (uint64_t)tid * kSeg;
            seg[j].load(in, pos, p.n);
            uint32_t nxt = __shfl_down(seg[j].at(0), 1, 64);
            if (lane == 63) nxt = (pos + 16 < p.n) ? Seg<InT>::load1(in, pos + 16) : 0u;
            uint32_t m = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                uint32_t a = seg[j].at(k);
                uint32_t b = k < 15 ? seg[j].at(k + 1) : nxt;
                uint32_t v = 0;
                bool hit;
                if constexpr (kDense) {
                    v = s_tab[swz_index(a, b)];
                    hit = (p.sentinel > 0xFFFFu) || (v != p.sentinel);
                } else {
                    // tokens are big-endian in memory; the key is the two u16 words as stored, the
                    // value comes back big-endian
                    const uint32_t key = a | (b << 16);
                    uint32_t r;
                    if constexpr (kHashLds) r = bucket_get(p, (const uint2*)s_hash, key);
                    else r = bucket_get(p, p.hbuckets, key);
                    hit = (r >> 31) != 0u;
                    v = r & 0xFFFFu;
                }
                m |= (uint32_t)hit << k;
                if (k & 1) vals[j][k >> 1] |= v << 16; else vals[j][k >> 1] = v;
            }
            // valid positions and right neighbours inside the buffer
            const uint32_t vmask = pos >= p.n ? 0u : (p.n - pos >= 16 ? 0xFFFFu : ((1u << (uint32_t)(p.n - pos)) - 1u));
            m &= (vmask >> 1) | (pos + 16 < p.n ? 0x8000u : 0u);
            // no merge across a chunk end: clear m at b - 1 for chunk starts b in (sub0, sub0 + kSubPos]
            if (nb < (uint32_t)kThreads) {   // (uniform) this lane's chunk starts b in [pos + 1, pos + 16]
                const uint32_t lo = (uint32_t)(pos - tile0) + 1u;
                for (uint32_t a = bnd_lower(lo); a < nb; ++a) {
                    const uint32_t r = s_bnd[a];
                    if (r > lo + 15u) break;
                    m &= ~(1u << (r - lo));
                }
            } else {
                uint64_t kidx;
                uint64_t b = first_boundary(p, sub0 + 1 < p.n ? sub0 + 1 : p.n, kidx);
                while (b < p.n && b <= sub0 + kSubPos) {
                    uint64_t e = b - 1;
                    if (e >= pos && e < pos + 16) m &= ~(1u << (uint32_t)(e - pos));
                    b = next_boundary(p, kidx);
                    ++kidx;
                }
            }
            mm[j] = m;
            valid[j] = vmask;
            const uint32_t ident = m == 0xFFFFu;
            const uint32_t M1 = merges_for(m, 1u), M0 = merges_for(m, 0u);
            const uint32_t cnt1 = __popc(lands_for(M1, 1u, vmask));
            const uint32_t cnt0 = __popc(lands_for(M0, 0u, vmask));
            const uint32_t cout = ((M1 >> 15) & 1u) ^ 1u;
            WaveFn fn;
            resolve_wave(ident, cout, cnt0, cnt1, lane, hasb[j], bco[j], excl[j], fn);
            if (lane == 0) s_wfn[j * kWaves + wave] = fn;
        }
        __syncthreads();

        // ---- phase 2: tile function, publish, look-back ----------------------------------
        if (wave == 0) {
            uint32_t gi = 0, gco = 0, g0 = 0, g1 = 0;
            if (lane < kGroupsT) { WaveFn f = s_wfn[lane]; gi = f.ident; gco = f.cout; g0 = f.cnt0; g1 = f.cnt1; }
            else { gi = 1; }
            uint32_t ghb, gbc, gex;
            WaveFn tf;
            // group counts fit 16 bits each (<= 1024 per group, <= 32768 per tile)
            resolve_wave(gi, gco, g0, g1, lane, ghb, gbc, gex, tf);
            if (lane < kGroupsT) {
                s_gin[lane][0] = ghb ? gbc : 0u;
                s_gin[lane][1] = ghb ? gbc : 1u;
                s_gin[lane][2] = gex & 0xFFFFu;
                s_gin[lane][3] = gex >> 16;
            }
            const uint32_t co0 = tf.ident ? 0u : tf.cout, co1 = tf.ident ? 1u : tf.cout;
            uint32_t C; uint64_t O;
            uint32_t how = 0xFFFFu;
            if (T == 0) {
                C = 1u; O = 0ull;
            } else {
                if (lane == 0) st_publish(p.status + T, st_agg(co0, co1, tf.cnt0, tf.cnt1));
                lookback(p, T, C, O, how);
            }
            if (lane == 0) {
                uint64_t end = O + (C ? tf.cnt1 : tf.cnt0);
                // invariant: a position emits at most one token; a failed tile writes nothing
                // (C = 2) and publishes a prefix only so its successors finish
                if (C > 1u || O > tile0 || end > p.n) {
                    if (C <= 1u) record_error(p, 4u, T, 0xFFu, O, end, C);
                    O = 0; C = 2u; end = 0;
                }
                st_publish(p.status + T, st_incl(C == 1u ? co1 : co0, end));
                s_C = C; s_O = O;
                if (p.debug) {
                    uint64_t* d = p.debug + 4ull * T;
                    d[0] = O;
                    d[1] = ((uint64_t)C << 32) | how;
                    d[2] = ((uint64_t)tf.cnt1 << 32) | tf.cnt0;
                    d[3] = ((uint64_t)co1 << 32) | co0;
                }
                s_tfn[2] = tf.cnt0; s_tfn[3] = tf.cnt1;
                if (T == p.ntiles - 1) {
                    *p.total = end;
                    if (p.chunk_off) p.chunk_off[p.nchunks] = end;
                    if (!kDense && p.done && end == p.n) *p.done = p.pass_id;   // no merge: the fixpoint
                }
            }
        }
        __syncthreads();

        // ---- phase 3: compact and store, one sub-tile at a time ---------------------------
        if (s_C > 1u) continue;   // failed tile (flagged): no output
        const uint32_t C = s_C;
        const uint64_t O = s_O;
        const uint32_t tile_cnt = C ? s_tfn[3] : s_tfn[2];
#pragma unroll
        for (int j = 0; j < kSubT; ++j) {
            const uint64_t sub0 = tile0 + (uint64_t)j * kSubPos;
            const uint64_t pos = sub0 + (uint64_t)tid * kSeg;
            const int g = j * kWaves + wave;
            const uint32_t cg = s_gin[g][C];
            const uint32_t og = s_gin[g][2 + C];
            const uint32_t c = hasb[j] ? bco[j] : cg;
            const uint32_t lane_off = og + (cg ? (excl[j] >> 16) : (excl[j] & 0xFFFFu));
            const uint32_t sub_first = s_gin[j * kWaves][2 + C];
            const uint32_t sub_end = (j + 1 < kSubT) ? s_gin[(j + 1) * kWaves][2 + C] : tile_cnt;
            const uint64_t gb = 2ull * (O + sub_first), ge = 2ull * (O + sub_end);
            const uint64_t ab = gb & ~15ull;
            const uint32_t M = merges_for(mm[j], c);
            const uint32_t L = lands_for(M, c, valid[j]);
            uint16_t* st16 = reinterpret_cast<uint16_t*>(s_stage);
            uint32_t r = (uint32_t)((2ull * (O + lane_off) - ab) >> 1);
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if ((L >> k) & 1u) {
                    uint32_t v = (vals[j][k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                    if constexpr (kDense) {
                        const uint32_t tok = ((M >> k) & 1u) ? v : seg[j].at(k);
                        st16[r++] = (uint16_t)(kBE ? bswap16(tok) : tok);
                    } else {   // u16 input and table values are already big-endian
                        st16[r++] = (uint16_t)(((M >> k) & 1u) ? v : seg[j].at(k));
                    }
                }
            }
            // token offsets of chunk starts in this segment
            if (p.chunk_off && nb < (uint32_t)kThreads) {   // this lane's chunk starts in [pos, pos + 16)
                const uint32_t lo = (uint32_t)(pos - tile0);
                for (uint32_t a = bnd_lower(lo); a < nb; ++a) {
                    const uint32_t r = s_bnd[a];
                    if (r > lo + 15u) break;
                    const uint32_t before = __popc(L & ((1u << (r - lo)) - 1u));
                    p.chunk_off[bk0 + a] = O + lane_off + before;
                }
            } else if (p.chunk_off) {
                uint64_t kidx;
                uint64_t b = first_boundary(p, sub0 < p.n ? sub0 : p.n, kidx);
                while (b < p.n && b < sub0 + kSubPos) {
                    if (b >= pos && b < pos + 16 && kidx < p.nchunks) {
                        uint32_t before = __popc(L & ((1u << (uint32_t)(b - pos)) - 1u));
                        p.chunk_off[kidx] = O + lane_off + before;
                    }
                    b = next_boundary(p, kidx);
                    ++kidx;
                }
            }
            __syncthreads();
            if (ge > p.out_cap || gb > ge) {
                if (tid == 0) record_error(p, 2u, T, (uint32_t)j, O, ge, C);
                __syncthreads();
                continue;
            }
            const uint32_t nblk = (uint32_t)((ge - ab + 15) >> 4);
            const uint4* st4 = reinterpret_cast<const uint4*>(s_stage);
            for (uint32_t i = tid; i < nblk; i += kThreads) {
                const uint64_t B = ab + 16ull * i;
                if (B >= gb && B + 16 <= ge) {
                    *reinterpret_cast<uint4*>(out + B) = st4[i];
                } else {
                    for (int u = 0; u < 8; ++u) {
                        const uint64_t bb = B + 2ull * u;
                        if (bb >= gb && bb < ge) *reinterpret_cast<uint16_t*>(out + bb) = st16[(bb - ab) >> 1];
                    }
                }
            }
            __syncthreads();
        }
    }
    if constexpr (kDense) self_reset(p, p.ntiles, &s_ticket);   // byte input: single-pass maps and pass 1
}

template <typename InT, bool kBE>
__global__ __launch_bounds__(kThreads) void merge_pass_kernel(PassParams p) {
    merge_pass_body<InT, kBE, false>(p);
}
// u16 passes (measured: one sub-tile per tile at 128 VGPRs, 4 waves per SIMD, is 45 % slower:
// the per-tile barriers and look-back dominate)
template <bool kHashLds>
__global__ __launch_bounds__(kThreads) void merge_tokens_kernel(PassParams p) {
    merge_pass_body<uint16_t, true, kHashLds>(p);
}

// ===========================================================================================
// Byte-input pass (the hot path: every map loaded from a merges file).
//
// Geometry: a workgroup of kThreads lanes takes a tile of kS sub-tiles; in a sub-tile lane l
// of wave w owns 16 consecutive positions (one 16-byte load), so a wave owns 1024 contiguous
// positions and emits them as one contiguous run of tokens.
//
// Self-token table: the LDS entry of a byte pair (a, b) is its merged token when (a, b) is a
// merge and the token of a itself otherwise (in output byte order).  A lookup then yields the
// token position i emits if it lands, and m[i] = (entry != token of a): one bit-op per two
// positions.  This needs no key (a, b) to map to a, which the host checks (self_ok); a
// position whose merge is cut (chunk end, buffer end) gets its raw byte patched in.
//
// Phase 1 (no synchronisation): per lane, 16 lookups, then the 16-bit merge mask is scanned
// under BOTH carry-in hypotheses at once — carry 0 in the low 16 bits, carry 1 in the high 16
// bits of one register, packed 16-bit adds/shifts (merges_for).  A wave resolves its lanes'
// carries with two ballots and one packed DPP prefix sum.
//
// Emission is deferred by one tile.  Iteration i runs phase 1 of tile T_i while wave 0 has
// the look-back loads of the previous tile T_{i-1} in flight; after phase 1 wave 0 resolves
// T_{i-1}'s carry-in and offset (its predecessors published their functions about one tile
// of work earlier, so the look-back rarely waits), a barrier, then the last wave resolves and
// publishes T_i's function while every wave writes T_{i-1}'s tokens: each lane writes one u16
// per position into its wave's LDS stage (a consumed position writes the slot the next,
// landing, position overwrites), and the wave copies the stage out with 16-byte buffer
// stores; as a sub-tile is written its input registers are refilled with the next tile's
// bytes.  The look-back reads a window of 64 status words per round trip and folds it with
// ballots and a wave sum.
// ===========================================================================================
namespace seg {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t pk_shl1(uint32_t v) {
    const u16x2 r = __builtin_bit_cast(u16x2, v) << (u16x2){1, 1};            // v_pk_lshlrev_b16
    return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) {
    const u16x2 r = __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b);   // v_pk_add_u16
    return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t pk_mul(uint32_t a, uint32_t b) {
    const u16x2 r = __builtin_bit_cast(u16x2, a) * __builtin_bit_cast(u16x2, b);   // v_pk_mul_lo_u16
    return __builtin_bit_cast(uint32_t, r);
}
// Each 16-bit half -> 1 if nonzero, else 0 (the compiler would expand min into compares).
__device__ __forceinline__ uint32_t pk_nz(uint32_t v) {
    uint32_t r;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(v), "s"(0x00010001u));
    return r;
}

typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef uint32_t __attribute__((aligned(2))) u32_a2;   // LDS takes 2-byte aligned u32 stores (gfx950)
typedef __attribute__((address_space(3))) u32_a2 lds_u32_a2;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
// LDS byte address of a __shared__ object.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const lds_u8*)(p);
}
// LDS byte addresses of the u16 entries at the low / high 16-bit index of t: base + 2 idx,
// one v_mad_u32_u16 each (op_sel picks the high half).
__device__ __forceinline__ uint32_t tab_addr_lo(uint32_t t, uint32_t base) {
    uint32_t a;
    asm("v_mad_u32_u16 %0, %1, 2, %2" : "=v"(a) : "v"(t), "s"(base));
    return a;
}
__device__ __forceinline__ uint32_t tab_addr_hi(uint32_t t, uint32_t base) {
    uint32_t a;
    asm("v_mad_u32_u16 %0, %1, 2, %2 op_sel:[1,0,0,0]" : "=v"(a) : "v"(t), "s"(base));
    return a;
}
// (No ds_read_u16_d16_hi here: with SRAM-ECC on, gfx950 d16 loads zero the other half.)
// a += 2 * bit, kept as one v_lshl_add (the compiler would re-derive each address from a count).
__device__ __forceinline__ void add2(uint32_t& a, uint32_t bit) {
    asm("v_lshl_add_u32 %0, %1, 1, %0" : "+v"(a) : "v"(bit));
}

// Workgroup geometry: 16 waves (4 per SIMD, 128 VGPRs each) times 2 sub-tiles per wave make one
// 32 KiB tile.
constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr int kS = 2;                                  // sub-tiles per tile
// Cache policy (buffer aux bits) of the input loads and the output stores: nt (2).  Every input
// byte is read once by one CU and every output byte written once: cfg3 0.604-0.613 -> 0.597-0.599 ms,
// cfg5 0.815-0.818 -> 0.804 ms (config_rates, same box); cfg2's 100 MiB, replayed back to back,
// loses its cache residency (0.0937 -> 0.0955 ms).
constexpr int kLdPol = 2, kStPol = 2;
constexpr uint32_t kWavePos = 64u * 16u;               // positions per wave per sub-tile
constexpr uint64_t kSubPos = (uint64_t)kWaves * kWavePos;
constexpr int kGroups = kS * kWaves;
// Per-wave token stage: a wave range of 1024 positions emits 512..1024 tokens; the stage holds
// 761 (2-byte aligned start + up to 1522 bytes), all the LDS the table leaves: every range of text
// or random bytes under a large merge map (~580 tokens).  A range with more tokens goes through it
// in two parts of 32 lanes (at most 512 tokens each).
constexpr int kStageWave = 1536;    // the LDS the table leaves, shared by the waves
// Look-back windows of 64 status words per round trip.  (Measured: 2 or 4 windows cost more
// through register spills than the extra round trips they save.)
constexpr int kLbWin = 1;
constexpr uint32_t kNone = 0xFFFFFFFFu;
static_assert(kSubPos * kS == kTilePosBytes, "tile geometry");
static_assert(kWavePos <= kMinChunkBytes, "at most one chunk end per wave sub-tile");
static_assert(kGroups <= 64, "one lane per group in the tile resolve");
static_assert(kStageWave % 16 == 0, "stage alignment");
static_assert((uint64_t)kS * kSubPos == kTilePosBytes, "tile = kS sub-tiles");

__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

// Buffer resource over base[0, left) (records clamped to 2^31 - 1): out-of-range loads return
// 0 and out-of-range stores are dropped.  Built from wave-uniform values only, so the accesses
// need no waterfall loop (cdna guide T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_at(const void* base, uint64_t left) {
    const uint32_t records = uni((uint32_t)(left > 0x7FFFFFFFull ? 0x7FFFFFFFull : left));
    const uint64_t addr = uni64((uint64_t)(uintptr_t)base);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((uintptr_t)addr), (short)0, (int)records,
                                             0x00020000);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t* in, uint64_t base, uint64_t n) {
    return rsrc_at(in + (base < n ? base : 0), base < n ? n - base : 0);
}

template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {   // lanes without a source read 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xF, false);
}
// Inclusive wave-wide prefix sum: row_shr 1/2/4/8 within rows, then row_bcast 15 and 31.
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {
    v += dpp0<0x111>(v);
    v += dpp0<0x112>(v);
    v += dpp0<0x114>(v);
    v += dpp0<0x118>(v);
    v += dpp0<0x142, 0xA>(v);
    v += dpp0<0x143, 0xC>(v);
    return v;
}
// mask's bit for this lane ? if1 : if0, one v_cndmask on the SGPR lane mask
__device__ __forceinline__ uint32_t lane_sel(uint64_t mask, uint32_t if0, uint32_t if1) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(mask));
    return r;
}
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int i) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, i);
}

// Phase-1 state of one tile of NS sub-tiles, per lane.
template <int NS>
struct TileStateT {
    uint32_t v[NS][8];   // looked-up tokens, two per register
    uint32_t mv[NS];     // merge mask | valid mask << 16
    uint32_t ex[NS];     // per wave carry-in h (h = 0: bits 0..15, h = 1: bits 16..31): the lane's
                         // exclusive prefix count (bits 0..14) and its carry-in (bit 15)
};
using TileState = TileStateT<kS>;

// ---- per-tile scalars ---------------------------------------------------------------------
struct TInfo {
    uint32_t rn;    // positions left in the buffer from the tile start (clamped to 2^31 - 1)
    uint32_t bge;   // first chunk start >= the tile start, relative (clamped to kFarPos)
    uint64_t k0;    // its chunk index
};

// The chunk geometry of tile T (every wave computes it for its own tiles: SALU work, no LDS).
// When the chunk size is a whole number of tiles (every chunk size of the configs: 16 MiB = 512
// tiles), T / (cs / tile) by a 32-bit high multiply with the host's reciprocal and at most two
// corrections; otherwise tile0 / cs by a 64-bit high multiply.
// "No chunk start in this tile or the first wave range after it": two tiles from the tile start
// (chunk starts and chunk sizes are capped there, so a range's one-past-the-end test never fires).
constexpr uint32_t kFarPos = 2u * (uint32_t)kTilePosBytes;
__device__ __forceinline__ TInfo tile_info(const PassParams& p, uint32_t T) {
    TInfo t;
    const uint64_t tile0 = (uint64_t)T * kTilePosBytes;
    const uint64_t left = p.n > tile0 ? p.n - tile0 : 0;
    t.rn = (uint32_t)(left > 0x7FFFFFFFull ? 0x7FFFFFFFull : left);
    if (p.cs_tiles) {
        const uint32_t d = p.cs_tiles;
        uint32_t q = d == 1u ? T : __umulhi(T, p.cs_tiles_magic);
        uint32_t r = T - q * d;
        if (r >= d) { q += 1u; r -= d; }
        if (r >= d) { q += 1u; r -= d; }
        const uint32_t left_tiles = r ? d - r : 0u;   // tiles to the next chunk start
        t.bge = left_tiles > 2u ? kFarPos : left_tiles * (uint32_t)kTilePosBytes;
        t.k0 = (uint64_t)q + (r ? 1u : 0u);
        return t;
    }
    const uint64_t cs = KARG(cs);   // (this path only: chunk sizes that are no whole number of tiles)
    uint64_t q = __umul64hi(tile0, KARG(cs_magic));
    uint64_t r = tile0 - q * cs;
    if (r >= cs) { q += 1; r -= cs; }
    if (r >= cs) { q += 1; r -= cs; }
    const uint64_t d = r ? cs - r : 0;
    t.bge = (uint32_t)(d > kFarPos ? kFarPos : d);
    t.k0 = q + (r ? 1u : 0u);
    return t;
}

// Lane functions (both carry-in hypotheses, packed 16-bit) and wave resolves of NS sub-tiles
// from their final merge masks m; the sub-tiles' dependency chains (ballots, SGPR carry chain,
// DPP scan) sit in one basic block so they interleave, and lane 63 writes every wave function
// (group g = j * kWaves + wave) after them.
template <int NS>
__device__ __forceinline__ void lane_wave_fns(const uint32_t (&m)[NS], uint32_t wave, int lane, TileStateT<NS>& st,
                                              uint32_t (*wfn)[4], uint32_t wlive = 0u) {
    uint64_t wnonid[NS], wcmask[NS];
    uint32_t wincl[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) wnonid[j] = __ballot(m[j] != 0xFFFFu);   // lanes that are not identities
#pragma unroll
    for (int j = 0; j < NS; ++j) {
#ifndef BLT_NO_DENSE_FNS
        if (wnonid[j] == 0) {
            // (uniform) a dense wave range: every position of every lane merges (and is valid: a
            // lane with a cut merge or an invalid position is no identity), as on text under a large
            // merge map.  Every lane is an identity and takes the wave's carry-in; under either it
            // emits 8 tokens (positions 0, 2, .., 14 or 1, 3, .., 15), so its exclusive count is
            // 8 lane under both hypotheses and the wave emits 512.  Carry-in bits: 0 under wave
            // carry-in 0, 1 under 1.  (The general path below derives the same words in ~30 VALU and
            // ~10 SALU instructions per wave range.)
            st.ex[j] = (uint32_t)lane * 0x00080008u | 0x80000000u;
            wcmask[j] = 0;
            wincl[j] = 0x02000200u;
            continue;
        }
#endif
        const uint32_t vm = st.mv[j] >> 16;
        const uint32_t mc = (m[j] & ~1u) | (m[j] << 16);
        const uint32_t sst = mc & ~pk_shl1(mc);
        const uint32_t rodd = mc & ~pk_add(mc, sst & 0xAAAAAAAAu);
        const uint32_t M = (mc & ~rodd & 0x55555555u) | (rodd & 0xAAAAAAAAu);
        const uint32_t L = ~(pk_shl1(M) | 1u) & (vm | (vm << 16));
        const uint32_t cnt0 = __popc(L & 0xFFFFu), cnt1 = __popc(L >> 16);
        // Carries across the wave, on SGPR masks: a lane's carry-in is the carry-out of the
        // nearest non-identity lane below it (an identity lane merges all 16 positions), or
        // the wave's carry-in c.  Y = lanes fed carry 1 by such a lane: each D = (non-identity,
        // carry-out 1) lane's carry runs up through the identity lanes above it and stops at
        // the next non-identity lane, i.e. the carry chain of M + (D << 1); F = lanes at or below
        // the lowest non-identity lane, fed by c.
        const uint64_t nonid = wnonid[j];
        const uint64_t cmask = __ballot(((M >> 31) & 1u) == 0u);   // carry-out 1 (if not identity)
        const uint64_t D = cmask & nonid, Mi = ~nonid, A = D << 1;
        const uint64_t Y = ((Mi + A) ^ Mi ^ A) | A;
        const uint64_t F = nonid ? ((nonid & (0ull - nonid)) << 1) - 1ull : ~0ull;
        const uint64_t CI0 = Y, CI1 = Y | F;
        // per lane: count under its carry-in, for wave carry-in 0 (low half) and 1 (high half)
        const uint32_t packed = lane_sel(CI0, cnt0, cnt1) | (lane_sel(CI1, cnt0, cnt1) << 16);
        const uint32_t incl = wave_scan(packed);
        st.ex[j] = (incl - packed) | lane_sel(CI0, 0u, 0x8000u) | lane_sel(CI1, 0u, 0x80000000u);
        wcmask[j] = cmask;
        wincl[j] = incl;
    }
    if (lane == 63) {
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const uint32_t g = (uint32_t)j * kWaves + wave;
            const uint64_t nonid = wnonid[j];
            wfn[g][0] = (nonid == 0) | (wlive << 1);   // identity | live << 1
            wfn[g][1] = nonid ? (uint32_t)((wcmask[j] >> (63 - __clzll(nonid))) & 1ull) : 0u;
            wfn[g][2] = wincl[j] & 0xFFFFu;
            wfn[g][3] = wincl[j] >> 16;
        }
    }
}

// ---- phase 1 of a tile: lookups, lane functions, wave functions ------------------------------
// Three straight-line passes over the kS sub-tiles (lookups; the rare uniform fix-up of buffer
// and chunk ends; lane functions and wave resolves), so the scheduler can overlap sub-tiles.
// kMode (the merge test of a self-token entry): 0 (kHiM) a merge value is >= 256, so "merge" is the
// entry's high byte; 1 the entry differs from the token of a itself; 2 as 1, and merges valued their
// own first byte a are stored as (mark << 8) | a (mark: a high byte no merge value has), whose high
// byte is cleared once the test is done.  allm (uniform): every byte pair is a merge (a merges file
// listing all 65 536 pairs), whatever the entry.  kLive: the lane also reports whether one of its
// merges (surviving buffer and chunk ends) made a token below 256, the only key components of a
// map whose keys are byte pairs: a first pass with none is the fixpoint (see scan_bytes_kernel).
template <bool kBE, int kMode, bool kLive>
__device__ __forceinline__ void phase1_tile(uint32_t tab, const uint32_t (&x)[kS][4], const uint32_t (&nxt)[kS],
                                            const TInfo& ti, uint32_t cs32, uint32_t wave, int lane,
                                            TileState& st, uint32_t (*wfn)[4], uint32_t allm, uint32_t mark,
                                            uint64_t* sub = nullptr) {
    static_assert(kBE, "the byte pass writes big-endian tokens");
    static_assert(kMode >= 0 && kMode <= 2 && !(kLive && kMode == 0), "phase-1 mode");
    uint32_t m[kS];
#pragma unroll
    for (int j = 0; j < kS; ++j) {
        // right neighbour of position 15: next lane's first byte (wave_shl:1); lane 63 keeps
        // the "old" operand, the byte after the wave's range (byte 0 of nbw; bytes 1..3 unused)
        const uint32_t nbw = (uint32_t)__builtin_amdgcn_update_dpp((int)nxt[j], (int)x[j][0], 0x130, 0xF, 0xF, false);
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            uint32_t va, vb;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                // position k = 2h + e: bytes (x_k, x_k+1) as u16 lanes [x_k, x_k+1] (one perm), then
                // the entry's LDS byte address 516 x_k + 2 x_k+1 + tab (one dot2, kSelfRow layout)
                const int k = 2 * h + e;
                const uint32_t lo = x[j][k >> 2], hi = (k >> 2) < 3 ? x[j][(k >> 2) + 1] : nbw;
                const uint32_t sel = 0x0C000C00u | ((uint32_t)((k & 3) + 1) << 16) | (uint32_t)(k & 3);
                const uint32_t pr = __builtin_amdgcn_perm(hi, lo, sel);
                const uint32_t addr = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, pr),
                                                             (u16x2){(unsigned short)(2 * kSelfRow), 2}, tab, false);
                const uint32_t v = *(const lds_u16*)(uintptr_t)addr;
                if (e == 0) va = v; else vb = v;
            }
            st.v[j][h] = __builtin_amdgcn_perm(vb, va, 0x05040100u);   // va | vb << 16, one op
        }
        uint32_t m32 = 0;   // even positions in bits 0..14, odd positions in bits 16..30
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            uint32_t d;
            if (kMode == 0) {
                // a merge is a token >= 256, a itself < 256: the token's high byte (BE: low byte)
                d = st.v[j][h] & 0x00FF00FFu;
            } else {
                // token of a itself (positions 2h, 2h+1: bytes 2h, 2h+1 of the lane), BE (a << 8)
                const uint32_t xw = x[j][h >> 1];
                const uint32_t self = __builtin_amdgcn_perm(xw, xw, (h & 1) ? 0x030C020Cu : 0x010C000Cu);
                d = st.v[j][h] ^ self;
                if (kMode == 2) {
                    // a marked entry (BE high byte = mark) is the merge value a: clear the mark
                    const uint32_t keep = pk_nz((st.v[j][h] ^ mark) & 0x00FF00FFu);   // 1: not marked
                    st.v[j][h] &= pk_mul(keep, 0x00FF00FFu) | 0xFF00FF00u;
                }
            }
            m32 |= pk_nz(d) << (2 * h);
        }
        if (allm) m32 = 0x7FFF7FFFu;
        m[j] = (m32 & 0xFFFFu) | (m32 >> 15);
    }
    // buffer end and chunk ends (uniform per wave range; rare)
    uint32_t bnext = ti.bge;   // first chunk start > the wave range's first position
#pragma unroll
    for (int j = 0; j < kS; ++j) {
        const uint32_t wrel = (uint32_t)j * (uint32_t)kSubPos + wave * kWavePos;
        while (bnext <= wrel) bnext += cs32;   // uniform; kSubPos / 4096 steps at most
        const uint32_t rem = ti.rn > wrel ? ti.rn - wrel : 0u;
        const bool has_end = bnext - 1u - wrel < kWavePos;
        if (rem <= kWavePos || has_end) {
            const uint32_t l16 = lane16_here();
            const int32_t r = (int32_t)(rem > 2u * kWavePos ? 2u * kWavePos : rem) - (int32_t)l16;
            const uint32_t vmask = r >= 16 ? 0xFFFFu : (r <= 0 ? 0u : ((1u << r) - 1u));
            uint32_t mm = m[j] & ((vmask >> 1) | (r > 16 ? 0x8000u : 0u));
            uint32_t forced = (r >= 1 && r <= 16) ? (1u << (r - 1)) : 0u;   // the buffer's last position
            if (has_end) {                                                   // chunk end b - 1 here
                const uint32_t e = bnext - 1u - wrel - l16;
                if (e < 16u) { mm &= ~(1u << e); forced |= 1u << e; }
            }
            if (__ballot(forced != 0)) {   // a cut merge emits its raw byte
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    const uint32_t xw = x[j][h >> 1];
                    const uint32_t raw = __builtin_amdgcn_perm(xw, xw, kBE ? ((h & 1) ? 0x030C020Cu : 0x010C000Cu)
                                                                           : ((h & 1) ? 0x0C030C02u : 0x0C010C00u));
                    const uint32_t fm = (((forced >> (2 * h)) & 1u) ? 0x0000FFFFu : 0u) |
                                        (((forced >> (2 * h + 1)) & 1u) ? 0xFFFF0000u : 0u);
                    st.v[j][h] = (st.v[j][h] & ~fm) | (raw & fm);
                }
            }
            m[j] = mm;
            st.mv[j] = mm | (vmask << 16);
        } else {
            st.mv[j] = m[j] | 0xFFFF0000u;
        }
    }
    uint32_t wlive = 0;
    if (kLive) {   // a surviving merge whose token is below 256 (BE high byte 0)
        uint32_t lv = 0;
#pragma unroll
        for (int j = 0; j < kS; ++j) {
            uint32_t low32 = 0;   // as m32: even positions in bits 0..14, odd in 16..30
#pragma unroll
            for (int h = 0; h < 8; ++h) low32 |= (pk_nz(st.v[j][h] & 0x00FF00FFu) ^ 0x00010001u) << (2 * h);
            lv |= m[j] & ((low32 & 0xFFFFu) | (low32 >> 15));
        }
        wlive = __ballot(lv != 0u) != 0 ? 1u : 0u;
    }
    if (sub) {   // timing build: lookups and masks done
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        sub[0] = __builtin_amdgcn_s_memtime();
    }
    lane_wave_fns<kS>(m, wave, lane, st, wfn, wlive);
    if (sub) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        sub[1] = __builtin_amdgcn_s_memtime();
    }
}

// ---- tile resolve (one wave): group carries and offsets, tile function, publish -------------
// kLive (u16 scan kernel): the groups' live bits (wfn[g][0] bit 1) are ORed into the tile's
// status word and into tfn[0] bit 1.
template <int NG = kGroups, bool kLive = false, bool kFresh = false>
__device__ __forceinline__ void resolve_tile(const PassParams& p, uint32_t T, int lane_arg, const uint32_t (*wfn)[4],
                                             uint32_t (*gin)[4], uint32_t* tfn) {
    // kFresh: the lane index computed here (a hoisted lane * 16 LDS offset was spilled, and its
    // reload's vmcnt wait made the tile resolve wait for the next tile's loads)
    const int lane = kFresh ? (int)(lane16_here() >> 4) : lane_arg;
    uint32_t gi = 1, gco = 0, g0 = 0, g1 = 0;
    if (lane < NG) { gi = wfn[lane][0]; gco = wfn[lane][1]; g0 = wfn[lane][2]; g1 = wfn[lane][3]; }
    const uint32_t tlive = kLive ? (__ballot((gi >> 1) & 1u) != 0) : 0u;
    if (kLive) gi &= 1u;
    const uint64_t nonid = __ballot(!gi);
    const uint64_t cmask = __ballot(gco);
    const uint64_t below = nonid & ((1ull << (uint32_t)lane) - 1ull);
    const uint32_t hb = below != 0;
    const uint32_t bc = hb ? (uint32_t)((cmask >> (63 - __clzll(below))) & 1ull) : 0u;
    const uint32_t cin0 = hb ? bc : 0u, cin1 = hb ? bc : 1u;
    uint32_t exc0, exc1, tot0, tot1;
    if constexpr ((uint64_t)NG * kWavePos < 65536u) {
        // a tile has at most 32768 tokens per hypothesis: both fit one packed scan
        const uint32_t my = (cin0 ? g1 : g0) | ((cin1 ? g1 : g0) << 16);
        const uint32_t inc = wave_scan(my);
        const uint32_t exc = inc - my;
        exc0 = exc & 0xFFFFu; exc1 = exc >> 16;
        const uint32_t tot = lane_u32(inc, 63);
        tot0 = tot & 0xFFFFu; tot1 = tot >> 16;
    } else {   // 64 KiB tiles: up to 65536 tokens, one scan per hypothesis
        const uint32_t my0 = cin0 ? g1 : g0, my1 = cin1 ? g1 : g0;
        const uint32_t inc0 = wave_scan(my0), inc1 = wave_scan(my1);
        exc0 = inc0 - my0; exc1 = inc1 - my1;
        tot0 = lane_u32(inc0, 63); tot1 = lane_u32(inc1, 63);
    }
    if (lane < NG) {
        gin[lane][0] = cin0;
        gin[lane][1] = cin1;
        gin[lane][2] = exc0;
        gin[lane][3] = exc1;
    }
    const uint32_t tident = nonid == 0;
    const uint32_t tcout = nonid ? (uint32_t)((cmask >> (63 - __clzll(nonid))) & 1ull) : 0u;
    const uint32_t co0 = tident ? 0u : tcout, co1 = tident ? 1u : tcout;
    if (lane == 0) {
        tfn[0] = co0 | (tlive << 1); tfn[1] = co1; tfn[2] = tot0; tfn[3] = tot1;
        // tile 0 starts with carry 1 at offset 0: its inclusive prefix is known at once
        st_publish(p.status + T, T == 0 ? st_incl(co1, tot1) | (tlive ? kStLiveIncl : 0ull)
                                        : st_agg(co0, co1, tot0, tot1) | (tlive ? kStLiveAgg : 0ull));
    }
}

// ---- look-back (wave 0) ------------------------------------------------------------------
// Lane l of window q reads the status of tile k - l - 64 q; tiles before 0 read as an
// inclusive prefix with carry 1 at offset 0.
// kFresh (the u16 scan kernel): 32-bit tile indices and the lane index computed here.  Hoisted out
// of its loop as 64-bit per-lane constants they were spilled to scratch, and every look-back
// waited for the reload's vmcnt, i.e. for the next tile's loads too (measured: f2 rows 1.5-3 %
// faster without; the byte pass, which does not spill them, 1 % slower with it).
template <bool kFresh = false>
__device__ __forceinline__ void lb_issue(const PassParams& p, int64_t k, int lane, uint64_t (&s)[kLbWin]) {
    if constexpr (kFresh) {
        const int32_t l = (int32_t)(lane16_here() >> 4);
#pragma unroll
        for (int q = 0; q < kLbWin; ++q) {
            const int32_t idx = (int32_t)k - l - 64 * q;
            s[q] = idx >= 0 ? st_read(p.status + (uint32_t)idx) : st_incl(1u, 0ull);
        }
    } else {
#pragma unroll
        for (int q = 0; q < kLbWin; ++q) {
            const int64_t idx = k - lane - 64 * q;
            s[q] = idx >= 0 ? st_read(p.status + idx) : st_incl(1u, 0ull);
        }
    }
}

// Function of the aggregates in lanes [0, lim) of one window (lane 0 newest) applied to
// carry-in c (into the oldest): returns the carry-out and adds the tokens to `tot`.
// kFresh (the u16 scan kernel): the lane index computed here (see lb_issue).
template <bool kFresh = false>
__device__ __forceinline__ uint32_t win_apply(uint64_t s, int lim, int lane_arg, uint32_t c, uint64_t& tot,
                                              uint32_t& live) {
    const int lane = lane_arg;   // (kFresh: see lb_issue; measured here it cost more spills)
    const bool in = lane < lim;
    live |= __ballot(in && (s & kStLiveAgg) != 0) != 0;
    const uint32_t hi = (uint32_t)(s >> 32), lo = (uint32_t)s;
    const uint32_t co0 = (hi >> 28) & 1u;
    const bool ident = ((hi >> 28) & 3u) == 2u;   // co0 = 0, co1 = 1
    const uint64_t inm = __ballot(in);
    const uint64_t nonid = __ballot(in && !ident);
    const uint64_t comask = __ballot(in && co0);   // a non-identity function is constant
    uint32_t cin;
    if (nonid == 0) {
        cin = c;                                   // identities only (dense text): c runs through
    } else if (nonid == inm) {
        // constants only (ordinary text): a lane's carry-in is the next older lane's carry-out;
        // the oldest lane in the window takes c
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp((int)co0, (int)co0, 0x130, 0xF, 0xF, false);
        cin = lane + 1 < lim ? up : c;
    } else {
        const uint64_t older = nonid & ~((~0ull) >> (63 - lane));
        cin = older ? (uint32_t)((comask >> __builtin_ctzll(older)) & 1ull) : c;
    }
    const uint32_t cnt = in ? (cin ? __builtin_amdgcn_alignbit(hi, lo, 30) & 0x1FFFFFFFu : lo & 0x3FFFFFFFu) : 0u;
    const uint32_t scan = wave_scan(cnt);
    tot += lane_u32(scan, 63);
    return nonid ? (uint32_t)((comask >> __builtin_ctzll(nonid)) & 1ull) : c;
}

struct TileFn {   // carry-in c -> (carry-out co_c, tokens t_c); selects, never indexed (no alloca)
    uint32_t co0, co1;
    uint64_t t0, t1;
};

// live: OR of the live bits of every tile before Tp (u16 scan kernel; 0 in the byte pass).
// Call it from wave-uniform control flow only (a branch on an SGPR value): its DPP scans
// (row_bcast) need the whole wave, and measured in a kernel that reached it through a branch on a
// VGPR value (finish_chunks_kernel's first version), the window sums came out wrong.
template <bool kFresh = false>
__device__ void lb_finish(const PassParams& p, uint32_t Tp, int lane, uint64_t (&s)[kLbWin], uint32_t& C,
                          uint64_t& O, uint32_t& how, uint32_t& spins, uint32_t& live, uint32_t* bad_out = nullptr) {
    TileFn acc = {0u, 1u, 0ull, 0ull};   // tiles between the windows read and Tp (identity)
    int64_t k = (int64_t)Tp - 1;
    uint32_t rounds = 0;
    SpinClock clk;
    for (;;) {
        int qs = -1, f = 64;
        bool ready = true;
#pragma unroll
        for (int q = 0; q < kLbWin; ++q) {
            const uint32_t flag = (uint32_t)(s[q] >> 62);
            const uint64_t inc = __ballot(flag == 2u), rdy = __ballot(flag != 0u);
            if (qs < 0) {
                if (inc) {
                    f = __builtin_ctzll(inc);
                    const uint64_t need = (~0ull) >> (63 - f);
                    if ((rdy & need) != need) ready = false;
                    qs = q;
                } else if (rdy != ~0ull) {
                    ready = false;
                }
            }
        }
        if (!ready && spins == 0 && bad_out) {   // debug: distance of the first tile not ready
            uint32_t d = 0;
#pragma unroll
            for (int q = kLbWin - 1; q >= 0; --q) {
                const uint64_t rdy = __ballot((uint32_t)(s[q] >> 62) != 0u);
                if (rdy != ~0ull) d = 64u * (uint32_t)q + (uint32_t)__builtin_ctzll(~rdy) + 1u;
            }
            *bad_out = d;
        }
        if (!ready) {
            ++spins;
            if (clk.expired()) {   // flagged; the tile writes nothing (C = 2)
                if (lane == 0) flag_error(p.ctl, KARG(sticky), 1u);
                C = 2u; O = 0ull;
                return;
            }
            __builtin_amdgcn_s_sleep(1);
            lb_issue<kFresh>(p, k, lane, s);
            continue;
        }
        if (qs < 0) {   // no inclusive prefix in 256 tiles: fold them into acc, read further back
            TileFn w;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint32_t c = (uint32_t)h;
                uint64_t t = 0;
#pragma unroll
                for (int q = kLbWin - 1; q >= 0; --q) c = win_apply<kFresh>(s[q], 64, lane, c, t, live);
                t += c ? acc.t1 : acc.t0;
                if (h == 0) { w.co0 = c ? acc.co1 : acc.co0; w.t0 = t; }
                else { w.co1 = c ? acc.co1 : acc.co0; w.t1 = t; }
            }
            acc = w;
            k -= 64 * kLbWin;
            ++rounds;
            lb_issue<kFresh>(p, k, lane, s);
            continue;
        }
        uint32_t c = 0;
        uint64_t off = 0;
#pragma unroll
        for (int q = kLbWin - 1; q >= 0; --q) {
            if (q > qs) continue;
            if (q == qs) {
                const uint64_t sf = ((uint64_t)lane_u32((uint32_t)(s[q] >> 32), f) << 32) | lane_u32((uint32_t)s[q], f);
                c = (uint32_t)(sf >> 61) & 1u;
                off = sf & (kStLiveIncl - 1ull);
                live |= (sf & kStLiveIncl) != 0;
                c = win_apply<kFresh>(s[q], f, lane, c, off, live);
            } else {
                c = win_apply<kFresh>(s[q], 64, lane, c, off, live);
            }
        }
        O = off + (c ? acc.t1 : acc.t0);
        C = c ? acc.co1 : acc.co0;
        how = (uint32_t)f | ((uint32_t)qs << 6) | (rounds << 8);
        return;
    }
}

// ---- dense wave ranges ----------------------------------------------------------------------
// Every pair of a wave range merges (text under a large merge map): every lane is an identity
// function, so all lanes take the wave's carry-in c and emit exactly 8 tokens - the low halves
// of v (c = 1, positions 0, 2, .., 14) or the high halves (c = 0, positions 1, 3, .., 15).  A lane
// packs them into 16 bytes.  Token n of the range goes to output byte rg + 2n past the 16-byte
// boundary ab, so the aligned block l holds the last rg/2 tokens of lane l-1 and the first
// 8 - rg/2 of lane l: one DPP fetch and a funnel shift per lane.
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t r) {
    return r ? __builtin_amdgcn_alignbyte(hi, lo, 2) : lo;   // r in {0, 2}
}
__device__ __forceinline__ u32x4 block_of(const u32x4& a, const u32x4& b, uint32_t d, uint32_t r) {
    // bytes [4d + r, 4d + r + 16) of the 32-byte concatenation a ++ b (d in 0..3, uniform)
    u32x4 o;
    if (d == 0) {
        o[0] = funnel(a[1], a[0], r); o[1] = funnel(a[2], a[1], r); o[2] = funnel(a[3], a[2], r); o[3] = funnel(b[0], a[3], r);
    } else if (d == 1) {
        o[0] = funnel(a[2], a[1], r); o[1] = funnel(a[3], a[2], r); o[2] = funnel(b[0], a[3], r); o[3] = funnel(b[1], b[0], r);
    } else if (d == 2) {
        o[0] = funnel(a[3], a[2], r); o[1] = funnel(b[0], a[3], r); o[2] = funnel(b[1], b[0], r); o[3] = funnel(b[2], b[1], r);
    } else {
        o[0] = funnel(b[0], a[3], r); o[1] = funnel(b[1], b[0], r); o[2] = funnel(b[2], b[1], r); o[3] = funnel(b[3], b[2], r);
    }
    return o;
}
// Dense wave range straight from registers: lane l's 16-byte output block goes
// to global memory with one buffer_store_b128, no LDS stage.  With the range 16-byte aligned
// (rg = 0: every tile of a dense text emits a multiple of 8 tokens) that is the whole emission;
// otherwise lane 0 stores the head of its block (its first 8 - rg/2 tokens) and lane 63 the block
// after the range (its last rg/2 tokens) token by token.
__device__ __forceinline__ void emit_dense(const uint32_t (&v)[8], uint32_t c, uint32_t rg, __amdgpu_buffer_rsrc_t ro,
                                           uint32_t ab, int lane) {
    const uint32_t sel = c ? 0x05040100u : 0x07060302u;   // low halves (c = 1) or high halves (c = 0)
    u32x4 P;
#pragma unroll
    for (int q = 0; q < 4; ++q) P[q] = __builtin_amdgcn_perm(v[2 * q + 1], v[2 * q], sel);
    const uint32_t o = ab + 16u * (uint32_t)lane;
    if (rg == 0) {
        __builtin_amdgcn_raw_buffer_store_b128(P, ro, (int)o, 0, kStPol);
        return;
    }
    u32x4 Q;   // lane l - 1's tokens
#pragma unroll
    for (int q = 0; q < 4; ++q)
        Q[q] = (uint32_t)__builtin_amdgcn_update_dpp((int)P[q], (int)P[q], 0x138, 0xF, 0xF, false);
    const uint32_t off = 16u - rg;
    if (lane != 0) __builtin_amdgcn_raw_buffer_store_b128(block_of(Q, P, off >> 2, off & 3u), ro, (int)o, 0, kStPol);
    if (lane == 0 || lane == 63) {
        const uint32_t h = 8u - (rg >> 1);   // tokens of this lane in its own block
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint16_t tok = (uint16_t)(P[k >> 1] >> (16 * (k & 1)));
            if (lane == 0 && (uint32_t)k < h) __builtin_amdgcn_raw_buffer_store_b16(tok, ro, (int)(ab + rg + 2u * k), 0, 0);
            if (lane == 63 && (uint32_t)k >= h)
                __builtin_amdgcn_raw_buffer_store_b16(tok, ro, (int)(ab + 1024u + 2u * (k - h)), 0, 0);
        }
    }
}

// ---- emission of the pending tile --------------------------------------------------------
// A lane's landed tokens into the stage at LDS byte address a, one u16 per position: a consumed
// position writes the slot the next landing token overwrites.  (Measured and rejected: one
// 2-byte-aligned u32 store per position pair, junk halves resolved by store order: bit-exact, but
// unaligned LDS stores run 2x slower on cfg5 and cfg2.)
__device__ __forceinline__ void stage_b16(const uint32_t (&v)[8], uint32_t L, uint32_t a) {
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        const uint32_t tok = v[h];
        *(lds_u16*)(uintptr_t)a = (uint16_t)tok;
        add2(a, __builtin_amdgcn_ubfe(L, 2 * h, 1));
        if (h < 7 || ((L >> 15) & 1u)) *(lds_u16*)(uintptr_t)a = (uint16_t)(tok >> 16);
        if (h < 7) add2(a, __builtin_amdgcn_ubfe(L, 2 * h + 1, 1));
    }
}

// Padded u16 stage (see kStageTok): logical byte x lives at x + 8 (x / 64).
__device__ __forceinline__ uint32_t stage_phys(uint32_t x) { return x + ((x >> 6) << 3); }
// stage_b16 into a padded stage: logical byte offset x from arr.
__device__ __forceinline__ void stage_b16_pad(const uint32_t (&v)[8], uint32_t L, uint8_t* arr, uint32_t x) {
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        const uint32_t tok = v[h];
        *reinterpret_cast<uint16_t*>(arr + stage_phys(x)) = (uint16_t)tok;
        add2(x, __builtin_amdgcn_ubfe(L, 2 * h, 1));
        if (h < 7 || ((L >> 15) & 1u)) *reinterpret_cast<uint16_t*>(arr + stage_phys(x)) = (uint16_t)(tok >> 16);
        if (h < 7) add2(x, __builtin_amdgcn_ubfe(L, 2 * h + 1, 1));
    }
}

// Copy-out of one stage part: whole 16-byte blocks (at most kCopyBlk per lane) and the head and
// tail fragments (u16 each, lanes 0..7 and 8..15).
constexpr int kCopyBlk = (kStageWave + 1023) / 1024;
// The u16 scan kernel has no 128 KiB table in LDS: its per-wave stage holds a whole wave range's
// tokens (a 2-byte aligned start and up to 1024 tokens), so every range goes out in one part.
// Few of its positions merge, so a lane's tokens fill ~32 bytes and the 32 lanes of a store write
// 4 banks (8-way conflicts).  The stage is padded: 8 bytes after every 64 (logical byte x lives at
// x + 8 (x / 64)), which spreads the lanes over the banks (2-way) and keeps 8-byte alignment for
// the copy-out's reads.  (Measured: u16 pass iteration 22.2 K -> 19.7 K cycles.)
constexpr int kStageTok = 2112;   // logical bytes per wave (>= 15 + 2048, a multiple of 64)
constexpr int kStageTokPhys = kStageTok / 64 * 72;   // physical bytes per wave
constexpr int kCopyBlkTok = (kStageTok + 1023) / 1024;
struct CopyPart {
    uint32_t abp;    // 16-byte aligned output byte of the part's first block (from obase)
    uint32_t rgp;    // the part's first token's byte offset from abp (0..15)
    uint32_t re;     // end of the part's tokens, from abp
};
template <int NB = kCopyBlk>
struct CopyData {
    u32x4 vb[NB];
    uint16_t vf;
};
// The byte pass's copy-out reads and stores run on every lane, with lanes that have nothing to
// store given an offset past the buffer (the store is dropped) instead of a branch around the
// instruction: a v_cndmask per instruction instead of an exec save / branch / restore (measured:
// cfg2 -1.5 %, cfg5 -0.5 %; the u16 pass's 3-block copy-out keeps its branches: kOob = false).
constexpr uint32_t kOobOff = 0x80000000u;   // >= every buffer resource's num_records (clamped to 2^31 - 1)
template <int NB>
__device__ __forceinline__ void copy_read(const uint8_t* stg, const CopyPart& c, int lane, CopyData<NB>& d) {
    const uint32_t hend = ((c.rgp + 15u) & ~15u) < c.re ? ((c.rgp + 15u) & ~15u) : c.re;
    const uint32_t tbeg = (c.re & ~15u) > hend ? (c.re & ~15u) : hend;
    const uint32_t nfull = (tbeg - hend) >> 4;
    const uint32_t of = lane < 8 ? c.rgp + 2u * (uint32_t)lane : tbeg + 2u * (uint32_t)(lane - 8);
    const bool bf = lane < 16 && of < (lane < 8 ? hend : c.re);
    const uint8_t* sp = stg;
    {   // unconditional LDS reads inside the workgroup's LDS (junk where not stored)
#pragma unroll
        for (int q = 0; q < NB; ++q)
            d.vb[q] = *reinterpret_cast<const u32x4*>(sp + min(hend + 16u * lane + 1024u * q, (uint32_t)kStageWave - 16u));
        d.vf = reinterpret_cast<const uint16_t*>(sp)[min(of >> 1, (uint32_t)kStageWave / 2u - 1u)];
        return;
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) {
        d.vb[q] = (u32x4){0u, 0u, 0u, 0u};
        if ((uint32_t)lane + 64u * q < nfull) d.vb[q] = *reinterpret_cast<const u32x4*>(sp + hend + 16u * lane + 1024u * q);
    }
    d.vf = bf ? reinterpret_cast<const uint16_t*>(sp)[of >> 1] : (uint16_t)0;
}
// copy_read from a padded stage (see kStageTok): the part starts at logical byte x0 of arr; a
// 16-byte block never crosses a 64-byte boundary, so it is two 8-byte aligned reads.
template <int NB>
__device__ __forceinline__ void copy_read_pad(const uint8_t* arr, uint32_t x0, const CopyPart& c, int lane, CopyData<NB>& d) {
    const uint32_t hend = ((c.rgp + 15u) & ~15u) < c.re ? ((c.rgp + 15u) & ~15u) : c.re;
    const uint32_t tbeg = (c.re & ~15u) > hend ? (c.re & ~15u) : hend;
    const uint32_t nfull = (tbeg - hend) >> 4;
    const uint32_t of = lane < 8 ? c.rgp + 2u * (uint32_t)lane : tbeg + 2u * (uint32_t)(lane - 8);
    const bool bf = lane < 16 && of < (lane < 8 ? hend : c.re);
#pragma unroll
    for (int q = 0; q < NB; ++q) {
        d.vb[q] = (u32x4){0u, 0u, 0u, 0u};
        if ((uint32_t)lane + 64u * q < nfull) {
            const uint8_t* b = arr + stage_phys(x0 + hend + 16u * lane + 1024u * q);
            const uint2 lo = *reinterpret_cast<const uint2*>(b), hi = *reinterpret_cast<const uint2*>(b + 8);
            d.vb[q] = (u32x4){lo.x, lo.y, hi.x, hi.y};
        }
    }
    d.vf = bf ? *reinterpret_cast<const uint16_t*>(arr + stage_phys(x0 + of)) : (uint16_t)0;
}
template <int NB, bool kOob = true>
__device__ __forceinline__ void copy_store(__amdgpu_buffer_rsrc_t ro, const CopyPart& c, int lane, const CopyData<NB>& d) {
    const uint32_t hend = ((c.rgp + 15u) & ~15u) < c.re ? ((c.rgp + 15u) & ~15u) : c.re;
    const uint32_t tbeg = (c.re & ~15u) > hend ? (c.re & ~15u) : hend;
    const uint32_t nfull = (tbeg - hend) >> 4;
    const uint32_t of = lane < 8 ? c.rgp + 2u * (uint32_t)lane : tbeg + 2u * (uint32_t)(lane - 8);
    const bool bf = lane < 16 && of < (lane < 8 ? hend : c.re);
    if (kOob) {
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const uint32_t o = (uint32_t)lane + 64u * q < nfull ? c.abp + hend + 16u * lane + 1024u * q : kOobOff;
            __builtin_amdgcn_raw_buffer_store_b128(d.vb[q], ro, (int)o, 0, kStPol);
        }
        __builtin_amdgcn_raw_buffer_store_b16(d.vf, ro, (int)(bf ? c.abp + of : kOobOff), 0, 0);
        return;
    }
#pragma unroll
    for (int q = 0; q < NB; ++q)
        if ((uint32_t)lane + 64u * q < nfull)
            __builtin_amdgcn_raw_buffer_store_b128(d.vb[q], ro, (int)(c.abp + hend + 16u * lane + 1024u * q), 0, kStPol);
    if (bf) __builtin_amdgcn_raw_buffer_store_b16(d.vf, ro, (int)(c.abp + of), 0, 0);
}

// Sparse wave range: per-lane landing mask and token offset, the range's token count.
struct SparseRange {
    uint32_t L, lane_off;   // per lane
    uint32_t gb, wcnt;      // uniform: output byte of the range (from obase), tokens
};

// Tile-level: carry-in C, O tokens before the tile; the output resource starts at the 16-byte
// boundary at or below byte 2 O, so every offset below is 32-bit.
__device__ __forceinline__ void emit_tile(const PassParams& p, uint32_t Tp, const TInfo& ti, uint32_t cs32,
                                          uint32_t wave, int lane, const TileState& st, const uint32_t (*gin)[4],
                                          uint32_t C, uint64_t O, uint8_t* stg, bool has_coff) {
    uint8_t* out = reinterpret_cast<uint8_t*>(KARG(out));   // (reloaded per tile: fewer live SGPRs)
    const uint64_t out_cap = KARG(out_cap);
    const uint64_t obase = (2ull * O) & ~15ull;
    const uint32_t orel = (uint32_t)(2ull * O - obase);
    const __amdgpu_buffer_rsrc_t ro = rsrc_at(out + obase, out_cap > obase ? out_cap - obase : 0);
    const uint32_t stg_lds = lds_addr(stg);
    uint32_t cnext = ti.bge;   // first chunk start >= the wave range's first position
    uint64_t kc = ti.k0;       // its chunk index
    SparseRange sr[kS];
    bool sparse[kS];
#pragma unroll
    for (int j = 0; j < kS; ++j) {
        const uint32_t g = (uint32_t)j * kWaves + wave;
        const uint32_t wrel = (uint32_t)j * (uint32_t)kSubPos + wave * kWavePos;
        const uint32_t cg = uni(gin[g][C]);
        const uint32_t goff = uni(gin[g][2 + C]);          // tokens before this wave range in the tile
        const uint32_t gb = orel + 2u * goff;              // output byte of the wave range, from obase
        // chunk start inside this wave range (cs >= 4096 > kWavePos: at most one)
        while (cnext < wrel) { cnext += cs32; ++kc; }   // uniform; kSubPos / 4096 steps at most
        const bool cstart = has_coff && cnext < ti.rn && cnext - wrel < kWavePos;
        sparse[j] = __ballot(st.mv[j] != 0xFFFFFFFFu) != 0;
        if (!sparse[j]) {
            // dense: every pair merges, no buffer end, so no chunk end: a chunk can only start at
            // the range's first position
            if (cstart && lane == 0) KARG(chunk_off)[kc] = O + goff;
            emit_dense(st.v[j], cg, gb - (gb & ~15u), ro, gb & ~15u, lane);
            continue;
        }
        const uint32_t m = st.mv[j] & 0xFFFFu, vmask = st.mv[j] >> 16;
        const uint32_t c = __builtin_amdgcn_ubfe(st.ex[j], 16u * cg + 15u, 1);
        const uint32_t lane_off = __builtin_amdgcn_ubfe(st.ex[j], 16u * cg, 15);
        const uint32_t mc = c ? m : (m & ~1u);
        const uint32_t sst = mc & ~(mc << 1);
        const uint32_t rodd = mc & ~(mc + (sst & 0xAAAAu));
        const uint32_t M = (mc & ~rodd & 0x5555u) | (rodd & 0xAAAAu);
        const uint32_t L = ~((M << 1) | (c ^ 1u)) & vmask;
        if (cstart) {
            const uint32_t e = cnext - wrel - lane16_here();
            if (e < 16u) KARG(chunk_off)[kc] = O + goff + lane_off + __popc(L & ((1u << e) - 1u));
        }
        sr[j].L = L;
        sr[j].lane_off = lane_off;
        sr[j].gb = gb;
        sr[j].wcnt = uni(lane_u32(lane_off + __popc(L), 63));
    }
    auto fits = [&](int j) { return (sr[j].gb & 15u) + 2u * sr[j].wcnt <= (uint32_t)kStageWave; };
#pragma unroll
    for (int j = 0; j < kS; ++j) {
        if (!sparse[j]) continue;
        // Stage -> global in one part, or in two (lanes 0..31, then 32..63: at most 512 tokens
        // each) when the range's tokens overflow the stage (few merges, e.g. random bytes).
        const uint32_t two = fits(j) ? 0u : 1u;
        const uint32_t off32 = two ? uni(lane_u32(sr[j].lane_off, 32)) : 0u;   // tokens before lane 32
        for (uint32_t part = 0; part <= two; ++part) {
            const uint32_t base = part ? off32 : 0u;
            const uint32_t cnt = two ? (part ? sr[j].wcnt - off32 : off32) : sr[j].wcnt;
            const uint32_t gbp = sr[j].gb + 2u * base;
            if (!two || ((uint32_t)lane >> 5) == part) {
                stage_b16(st.v[j], sr[j].L, stg_lds + (gbp & 15u) + 2u * (sr[j].lane_off - base));
            }
            const CopyPart cp = {gbp & ~15u, gbp & 15u, (gbp & 15u) + 2u * cnt};
            CopyData<> d;
            copy_read(stg, cp, lane, d);
            copy_store(ro, cp, lane, d);
        }
    }
}

// ---- refill: the bytes of tile Tn into x --------------------------------------------------
// Straight-line 16-byte loads through a descriptor clamped to whole dwords (a load must not
// reach past the buffer; a partly out-of-range load reads 0), then, only in the wave range
// holding the buffer end, the lanes' bytes again one by one.  Keeping the common path free of
// branches lets the loads land in x directly: a branch that merges x would make the compiler
// wait for them right here.
__device__ __forceinline__ void load_tile(const PassParams& p, uint32_t Tn, uint32_t wave, int lane,
                                          uint32_t (&x)[kS][4], uint32_t (&nxt)[kS]) {
    const uint8_t* in = reinterpret_cast<const uint8_t*>(KARG(in));   // (reloaded per tile)
    const uint64_t tile0 = (uint64_t)Tn * kTilePosBytes;
    const uint64_t left = p.n > tile0 ? p.n - tile0 : 0;
    const __amdgpu_buffer_rsrc_t r = rsrc_at(in + tile0, left);
    const __amdgpu_buffer_rsrc_t rd = rsrc_at(in + tile0, left & ~3ull);
    const uint32_t rn = (uint32_t)(left > 0x7FFFFFFFull ? 0x7FFFFFFFull : left);
#pragma unroll
    for (int j = 0; j < kS; ++j) {
        const uint32_t wrel = (uint32_t)j * (uint32_t)kSubPos + wave * kWavePos;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rd, (int)wrel + 16 * lane, 0, kLdPol);
        x[j][0] = v[0]; x[j][1] = v[1]; x[j][2] = v[2]; x[j][3] = v[3];
        // the byte after the range, as its whole (4-aligned) dword: a u8 load would be masked
        // right here, which makes the compiler wait for it.  The range check covers voffset
        // only, never soffset: offsets go in voffset.
        nxt[j] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rd, (int)(wrel + kWavePos), 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kS; ++j) {
        const uint32_t wrel = (uint32_t)j * (uint32_t)kSubPos + wave * kWavePos;
        if (rn > wrel && rn - wrel < kWavePos + 16u) {   // uniform: the buffer end is near this range
            nxt[j] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)(wrel + kWavePos), 0, 0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t d = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    d |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)wrel + 16 * lane + 4 * q + b, 0, 0)
                         << (8 * b);
                x[j][q] = d;
            }
        }
    }
}

// Workgroup-internal dataflow: monotonic LDS counters instead of block barriers, so waves drift
// (a fast wave starts the next phase while a slow one finishes) and phase-1 LDS reads, emission
// LDS writes and VALU work of different waves overlap.  Every wait names exactly one producer
// condition; rings of kRing slots cover the at most two iterations of drift the chain allows
// (a wave emits iteration i only after tile i-1 is resolved, which needs every wave's phase 1).
constexpr int kRing = 4;
// Per-wave phase stamps and look-back timing (tools/tile_timing.py) only in the timing build
// (-DBLT_TIMING): kept live across the loop they cost scalar registers the kernel has none of.
#ifdef BLT_TIMING
constexpr bool kTiming = true;
#else
constexpr bool kTiming = false;
#endif
// Wave priorities (s_setprio) during phase 1 and emission: waves >= k*Wave get k*.  The SIMD
// arbiter favours old waves, so without help the youngest waves finish phase 1 last (holding back
// the tile's resolve and the aggregate that other workgroups' look-backs wait for) and emission
// last (holding back their next phase 1); no priorities at all cost 20 %.
constexpr int kPrioP1Wave = kWaves / 2, kPrioP1 = 1;
constexpr int kPrioEmWave = 3 * kWaves / 4, kPrioEm = 2;
constexpr int kTkTid = 64;   // the lane that claims tickets and hands them over (wave 1)
__device__ __forceinline__ uint32_t lds_acquire(const uint32_t* f) {
    return __hip_atomic_load(const_cast<uint32_t*>(f), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(uint32_t* f, uint32_t v) {
    __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Waits until *f >= v; on a (never expected) timeout flags error bit 8 and lets the wave go on.
__device__ __forceinline__ void wait_ge(const PassParams& p, const uint32_t* f, uint32_t v) {
    SpinClock clk;
    while (lds_acquire(f) < v) {
        if (clk.expired()) {
            if ((threadIdx.x & 63) == 0) flag_error(p.ctl, KARG(sticky), 8u);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// The merge scan over a whole buffer (see the block comment of namespace seg).  Per iteration
// a workgroup holds three tiles: T (phase 1 now; its bytes were loaded during the previous
// iteration), Tp (pending emission: its carry-in and offset come from the look-back) and Tq (the
// next T: its bytes are loaded now, a whole iteration ahead).  The ticket after Tq is claimed
// at the start of the iteration by one lane (tid 64) and handed over at the end of the claiming
// wave's emission (a whole iteration for the device-scope atomic to return).  (Measured: the
// claiming lane computing the claimed tile's chunk geometry once for all waves and publishing it
// with the ticket delays the hand-over, and cfg3 loses 2 %.)
//
// kLive (the first pass of a general map whose keys are all byte pairs): the tiles' live bits (a
// merge made a token below 256: see phase1_tile) travel with the status words, and the last tile
// marks the pass final (done = kDoneBytePass) when no tile had one: every later pass would merge
// nothing (a pair this pass left alone was looked up and rejected; a token >= 256 is in no key),
// so the u16 passes the host enqueued behind it return at once.
template <bool kBE, int kMode, bool kLive>
__global__ __launch_bounds__(kThreads) void scan_bytes_kernel(PassParams p) {
    __shared__ __attribute__((aligned(16))) uint16_t s_tab[kSelfEntries];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[kWaves][kStageWave];
    __shared__ __attribute__((aligned(16))) uint32_t s_wfn[kRing][kGroups][4];   // wave functions (phase 1)
    __shared__ uint32_t s_gin[kRing][kGroups][4];   // group carry-in |H=0,1, offset |H=0,1
    __shared__ uint32_t s_tfn[kRing][4];            // tile co0, co1, tot0, tot1
    __shared__ uint64_t s_O[kRing];                 // tokens before the tile
    __shared__ uint32_t s_C[kRing];                 // carry into the tile (2: failed tile, no output)
    __shared__ uint32_t s_tk[kRing];        // claimed tickets
    __shared__ uint32_t s_p1cnt[kRing];     // phase-1 arrivals per slot (kWaves per use); waves
                                            // drift across iterations, so one counter would mix them
    __shared__ uint32_t s_rdone;            // iterations whose tile is resolved
    __shared__ uint32_t s_lbdone;           // iterations whose pending tile has C, O
    __shared__ uint32_t s_tkdone;           // iterations whose next ticket is in s_tk

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t wave = uni((uint32_t)tid >> 6);
    const uint64_t n = p.n;
    const uint32_t ntiles = p.ntiles;
    const uint32_t cs32 = (uint32_t)(p.cs > kFarPos ? kFarPos : p.cs);
    const uint32_t allm = uni(p.allm), mark = uni(p.mark);
    const bool has_coff = p.chunk_off != nullptr;   // (the pointer itself is reloaded where stored)

    const uint32_t cover = ws_cover(p);
    // timing build: workgroup start, table copied, exit (s_memrealtime) after the per-tile records
    uint64_t* const wg_rec = (kTiming && p.debug) ? p.debug + (8ull + 8ull * kWaves) * p.ntiles + 4ull * blockIdx.x : nullptr;
    if (wg_rec && tid == 0) wg_rec[0] = __builtin_amdgcn_s_memrealtime();
    // the tickets first: a claim waits for its atomic, and the next one is claimed a round trip
    // later (other workgroups' claims in between: measured, two consecutive tiles are slower)
    if (tid == 0) {
        s_tk[kRing - 2] = atomicAdd(p.ctl, 1u);   // T
        s_tk[kRing - 1] = atomicAdd(p.ctl, 1u);   // Tq, the tile after it
        for (int r = 0; r < kRing; ++r) s_p1cnt[r] = 0;
        s_rdone = 0; s_lbdone = 0; s_tkdone = 0;
    }
    {
        const uint4* src = reinterpret_cast<const uint4*>(p.dense);
        uint4* dst = reinterpret_cast<uint4*>(s_tab);
        // LDS-DMA, every load in flight at once (one wave-instruction fills 1 KiB of LDS).  (A
        // rolled copy loop waits for each load: one L2/MALL round trip each, ~0.7 us when all 256
        // workgroups copy at once, 6.9 us in all.  Round 6: the first tile's loads issued beside the
        // copy, the tickets handed over by an LDS-only barrier, measured cfg2 2 % slower.)
        constexpr int kUnits = (int)(kSelfEntries * 2 / 16);
        constexpr int kPer = (kUnits + kThreads - 1) / kThreads;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int u0 = (int)wave * 64 + k * kThreads;   // the wave's first unit (uniform)
            if (k < kPer - 1 || u0 < kUnits)
                __builtin_amdgcn_global_load_lds(
                    (__attribute__((address_space(1))) void*)(src + u0 + lane),
                    (__attribute__((address_space(3))) void*)(dst + u0), 16, 0, 0);
        }
    }
    __syncthreads();
    if (wg_rec && tid == 0) wg_rec[1] = __builtin_amdgcn_s_memrealtime();
    const uint32_t tab = uni(lds_addr(s_tab));
    uint32_t T = uni(s_tk[kRing - 2]);    // tile in phase 1
    uint32_t Tp = kNone;                  // tile waiting for emission
    uint32_t Tq = uni(s_tk[kRing - 1]);   // the tile after T (its bytes load during T's iteration)
    if (ws_refused(p, ntiles, cover)) T = kNone;   // (its two tickets are dropped: the reset zeroes them)
    if (T >= ntiles || Tq >= ntiles) Tq = kNone;
    TInfo ti = {}, tip = {};
    if (T < ntiles) ti = tile_info(p, T);
    __syncthreads();

    uint32_t xa[kS][4], xb[kS][4];   // input bytes of each sub-tile: T's, and Tq's (ping-pong)
    uint32_t na[kS], nb[kS];         // byte after each wave range (lane 63's right neighbour)
    if (T < ntiles) load_tile(p, T, wave, lane, xa, na);
    TileState sa, sb;       // phase-1 states: T's and Tp's (ping-pong)
    uint64_t lbs[kLbWin];   // look-back wave: status words for the pending tile's look-back
    uint32_t it = 0;

    // One iteration: phase 1 of T from `x` into `sc`, emission of Tp from `sp`, Tq's bytes into
    // `xq`.  The loop runs it twice per trip with the roles swapped, so no state is copied.
    auto step = [&](uint32_t (&x)[kS][4], uint32_t (&nxt)[kS], uint32_t (&xq)[kS][4], uint32_t (&nxtq)[kS],
                    TileState& sc, const TileState& sp) {
        const uint32_t slot = it & (kRing - 1), pslot = (it - 1) & (kRing - 1);
        uint64_t stamp[7], sub[2] = {0, 0};
        const bool stamping = kTiming && p.debug != nullptr;
        if (stamping) stamp[0] = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): T's bytes have landed
        if (stamping) stamp[1] = __builtin_amdgcn_s_memtime();
        if (Tq < ntiles) load_tile(p, Tq, wave, lane, xq, nxtq);   // a whole iteration to land
        // the tile after Tq, claimed now: claimed one phase before its bytes are needed, so claim
        // order stays close to publish order (a tile claimed further ahead lands behind
        // later-claimed ones and stalls their look-backs)
        uint32_t tk = kNone;
        if (tid == kTkTid && Tq < ntiles) tk = atomicAdd(p.ctl, 1u);
        asm volatile("" ::: "memory");

        // ---- phase 1 of T; the last wave to finish it resolves and publishes T ----------------
        bool lbw = wave == 0;   // the wave that resolves Tp: the first to finish phase 1
        if (T < ntiles) {
            // issue priority by age: the youngest waves lose the arbiter to the older ones, finish
            // phase 1 last and so hold back the tile's resolve and aggregate (which successors'
            // look-backs wait for), and finish emission last (which holds back their next phase 1)
            if (wave >= (uint32_t)kPrioP1Wave) __builtin_amdgcn_s_setprio(kPrioP1);
            phase1_tile<kBE, kMode, kLive>(tab, x, nxt, ti, cs32, wave, lane, sc, s_wfn[slot], allm, mark,
                                           stamping ? sub : nullptr);
            __builtin_amdgcn_s_setprio(0);
            uint32_t old = 0;
            if (lane == 0)
                old = __hip_atomic_fetch_add(&s_p1cnt[slot], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
            old = uni(old);
            lbw = old == (uint32_t)kWaves * (it / kRing);
            if (old == (uint32_t)kWaves * (it / kRing + 1u) - 1u) {
                resolve_tile<kGroups, kLive, kMode != 0>(p, T, lane, s_wfn[slot], s_gin[slot], s_tfn[slot]);
                if (lane == 0) lds_release(&s_rdone, it + 1u);
                if (stamping && lane == 0) p.debug[4ull * ntiles + 4ull * T] = __builtin_amdgcn_s_memrealtime();
            }
        }
        if (stamping) stamp[2] = __builtin_amdgcn_s_memtime();

        // ---- carry-in and offset of Tp, by the first wave to finish phase 1: its snapshot is
        // the freshest that still lands before the slower waves finish (~0.5 us round trip)
        if (lbw && Tp < ntiles) {
            uint32_t C = 1u, how = 0xFFFFu, spins = 0, bad = 0, live = 0;
            uint64_t O = 0ull;
            const bool lb = Tp > 0;
            if (lb) lb_issue<kMode != 0>(p, (int64_t)Tp - 1, lane, lbs);
            const uint64_t rt_snap = stamping ? __builtin_amdgcn_s_memrealtime() : 0;
            // Tp was resolved last iteration: its tile function is read while the snapshot flies
            wait_ge(p, &s_rdone, it);
            const uint32_t tfl = uni(s_tfn[pslot][0]), tf1 = uni(s_tfn[pslot][1]);
            const uint32_t tf0 = tfl & 1u, tf2 = uni(s_tfn[pslot][2]), tf3 = uni(s_tfn[pslot][3]);
            if (lb) lb_finish<kMode != 0>(p, Tp, lane, lbs, C, O, how, spins, live, kTiming ? &bad : nullptr);
            live |= (tfl >> 1) & 1u;   // tiles up to and including Tp (kLive; 0 otherwise)
            if (lane == 0) {
                const uint64_t end = O + (C == 1u ? tf3 : tf2);
                // a failed tile (flagged) writes nothing (C = 2) and publishes a prefix only so its
                // successors finish
                if (C > 1u || O > (uint64_t)Tp * kTilePosBytes || end > n) {
                    if (C <= 1u) record_error(p, 4u, Tp, 0xFFu, O, end, C);
                    O = 0; C = 2u;
                }
                // the other waves need only C and O: release them first, publish after
                s_C[pslot] = C;
                s_O[pslot] = O;
                lds_release(&s_lbdone, it + 1u);
                const uint64_t fin = C > 1u ? 0ull : O + (C ? tf3 : tf2);
                if (Tp > 0) st_publish(p.status + Tp, st_incl(C == 1u ? tf1 : tf0, fin) | (live ? kStLiveIncl : 0ull));
                if (2ull * fin > KARG(out_cap)) record_error(p, 2u, Tp, 0xFFu, O, fin, C);
                if (Tp == ntiles - 1) {
                    *KARG(total) = fin;
                    if (uint64_t* co = KARG(chunk_off)) co[KARG(nchunks)] = fin;
                    if (kLive && C <= 1u && (fin == n || !live))
                        if (uint32_t* dn = KARG(done)) *dn = kDoneBytePass;
                }
                if (kDebugRecord && p.debug) {
                    uint64_t* d = p.debug + 4ull * Tp;
                    d[0] = O;
                    d[1] = ((uint64_t)C << 32) | how;
                    d[2] = ((uint64_t)tf3 << 32) | tf2;
                    d[3] = ((uint64_t)tf1 << 32) | tf0;
                    if (kTiming) {
                        uint64_t* e = p.debug + 4ull * ntiles + 4ull * Tp;
                        e[3] = spins | ((uint64_t)bad << 32);
                        e[1] = (rt_snap & 0xFFFFFFFFull) | (__builtin_amdgcn_s_memrealtime() << 32);
                    }
                }
            }
        }

        // ---- emission of Tp (T's bytes are consumed; Tq's loads fly meanwhile) ----------------
        if (stamping) stamp[3] = __builtin_amdgcn_s_memtime();
        if (Tp < ntiles) {
            wait_ge(p, &s_lbdone, it + 1u);
            if (stamping) stamp[4] = __builtin_amdgcn_s_memtime();
            if (wave >= (uint32_t)kPrioEmWave) __builtin_amdgcn_s_setprio(kPrioEm);
            const uint32_t Cp = uni(s_C[pslot]);
            if (Cp <= 1u)   // C = 2: a failed tile (flagged), no output
                emit_tile(p, Tp, tip, cs32, wave, lane, sp, s_gin[pslot], Cp, uni64(s_O[pslot]), s_stage[wave], has_coff);
            __builtin_amdgcn_s_setprio(0);
        }
        if (stamping) stamp[5] = __builtin_amdgcn_s_memtime();
        if (stamping && Tp < ntiles && lane == 0) {
            stamp[6] = __builtin_amdgcn_s_memtime();
            uint64_t* w = p.debug + 8ull * ntiles + 8ull * ((uint64_t)Tp * kWaves + wave);
#pragma unroll
            for (int q = 0; q < 6; ++q) w[q] = stamp[q + 1] - stamp[q];
            w[6] = sub[0] ? sub[0] - stamp[1] : 0;   // phase 1 split: lookups and masks | lane functions
            w[7] = sub[0] ? sub[1] - sub[0] : 0;
        }
        if (stamping && tid == 0 && Tp < ntiles) {
            uint64_t* e = p.debug + 4ull * ntiles + 4ull * Tp;
            e[2] = __builtin_amdgcn_s_memtime();
        }
        // Tq <- the ticket claimed at this iteration's start (handed over after the claiming
        // wave's emission); T <- Tq (its bytes were loaded during this iteration)
        if (tid == kTkTid) {
            s_tk[slot] = tk;
            lds_release(&s_tkdone, it + 1u);
        }
        uint32_t Tr = kNone;
        if (Tq < ntiles) {
            wait_ge(p, &s_tkdone, it + 1u);
            Tr = uni(s_tk[slot]);
            if (Tr >= ntiles) Tr = kNone;
        }
        tip = ti;
        if (Tq < ntiles) ti = tile_info(p, Tq);
        Tp = T;
        T = Tq;
        Tq = Tr;
        ++it;
    };
    for (;;) {
        if (!(T < ntiles || Tp < ntiles)) break;
        step(xa, na, xb, nb, sa, sb);
        if (!(T < ntiles || Tp < ntiles)) break;
        step(xb, nb, xa, na, sb, sa);
    }
    if (wg_rec && lane == 0)
        atomicMax(reinterpret_cast<unsigned long long*>(wg_rec + 2), (unsigned long long)__builtin_amdgcn_s_memrealtime());
    self_reset(p, ntiles, &s_tkdone);
}

// ===========================================================================================
// u16 passes of a general map (tokenizer.rs:63-86, every pass after the first) on the byte
// pass's structure: tickets, one tile in phase 1 while the previous one is looked back and
// emitted, barrier-free LDS counters.  The input is the previous pass's big-endian u16 tokens.
//
// Geometry: in sub-tile j lane l of wave w owns tokens [16384 j + 1024 w + 16 l, +16) of a tile
// (two 16-byte loads), so a tile is kSt = 2 sub-tiles of 16 wave ranges of 1024 tokens (64 KiB of
// input; measured: one sub-tile per tile, 0.65 ms for the 256 MiB multi-pass case against 0.61).
// A wave range's tokens go out through a per-wave stage that holds all of them (one part).
//
// Lookups: a 2-choice cuckoo table of 8-byte buckets [key, value] (the LDS when it fits, else
// global memory).  The key of the pair (a, b) is the pair's two u16 words as stored, so an even
// position's key is the lane's input dword itself and an odd one's is one alignbyte; a bucket is
// the top bits of one v_dot2_u32_u16 of the key with the host's multiplier pair; the value word
// is BE(v) | 1 << 31 | live << 30, so one byte permute turns two results into the pair's merge
// mask, and an OR of the results tells whether a merge made a key component ("live").
//
// Chunk ends: the chunk starts of this pass are the previous pass's chunk offsets.
// chunk_map_kernel turns them into one word per wave range (at most one chunk start and one
// chunk end in 1024 tokens: the host runs this kernel only while every chunk holds at least
// kTokRange tokens, i.e. chunk_size >> pass >= 1024).
//
// In place: the pass may write over its own input.  A tile writes only below the end of its
// own input, and only after its look-back, i.e. after every earlier tile published its
// aggregate, which each does after its own loads; so every byte a tile overwrites has been read.
// A wave range whose output is its input (no merge before it in the buffer and none in it)
// writes nothing, so a pass that merges nothing (the fixpoint check) only reads.
// ===========================================================================================
constexpr int kSt = (int)(kTilePosTok / kTokRange) / kWaves;   // sub-tiles per token tile (2 at 16 waves)
constexpr uint32_t kSubTok = (uint32_t)kWaves * kWavePos;   // tokens per sub-tile (16 wave ranges)
constexpr uint32_t kTileTok = (uint32_t)kSt * kSubTok;
constexpr int kGroupsTok = kSt * kWaves;
static_assert(kTileTok == kTilePosTok && kWavePos == kTokRange, "token tile geometry");
static_assert(kGroupsTok <= 64 && kS * kWaves <= 64, "groups");

// Chunk-map word of a wave range: bits 0..10 offset of a chunk start, bit 11 set if there is one;
// bits 12..22 offset of the last token of a chunk (a start minus one), bit 23 set if there is
// one; bits 32..63 the start's chunk index.
constexpr uint32_t kCmStart = 1u << 11, kCmEnd = 1u << 23;

// The next pass's chunk-map words for chunk c starting at output token P (round 6): the start in
// P's wave range, the end of chunk c - 1 in the range of P - 1.  The two marks of one word can come
// from two tiles on two XCDs: agent-scope ORs into a map zeroed one pass earlier.  (It replaces a
// chunk_map_kernel launch per u16 pass, 4.8 us plus its launch gap on the chain row.)  The host
// asks for the map only when the next pass runs on this kernel, so its chunks hold kTokRange tokens
// or more: a second start or end in one range is chunk_map_kernel's error 16 (host bug).
__device__ __forceinline__ void cm_mark(const PassParams& p, uint64_t* m, uint64_t P, uint32_t c) {
    const uint64_t o1 = __hip_atomic_fetch_or(m + (P >> 10), (P & 1023u) | kCmStart | ((uint64_t)c << 32),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t o2 = 0;
    if (c) o2 = __hip_atomic_fetch_or(m + ((P - 1) >> 10), (((P - 1) & 1023u) << 12) | kCmEnd, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    if ((o1 & kCmStart) || (o2 & kCmEnd)) flag_error(p.ctl, KARG(sticky), 16u);
}

__device__ __forceinline__ uint64_t token_count(const PassParams& p) {
    return p.n_dev ? __hip_atomic_load(const_cast<uint64_t*>(p.n_dev), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : p.n;
}
__device__ __forceinline__ bool pass_done(const PassParams& p) {
    return p.done && __hip_atomic_load(p.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

// One thread per wave range: lower bound of the range start in the chunk starts.  It also zeroes
// the scan's ticket and status words (one per kTileTok tokens, so the wave ranges cover them): the
// previous pass has finished with them.  The error flags and first-error record (ctl[1..]) stay,
// so the host reports the chain's first failure (the chain's first memset zeroed them).
// Chunk-map word of the wave range [lo, hi) from the sorted chunk starts cs[0, nc): lower bound
// of lo, the start inside the range and the end (a start minus one) inside it.
__device__ __forceinline__ uint64_t cm_word(const uint64_t* cs, uint64_t nc, uint64_t lo, uint64_t hi, bool& bad) {
    uint64_t a = 0, b = nc;
    while (a < b) {
        const uint64_t mid = (a + b) >> 1;
        if (cs[mid] < lo) a = mid + 1; else b = mid;
    }
    uint64_t w = 0;
    if (a < nc && cs[a] < hi) {
        w |= (cs[a] - lo) | kCmStart | (a << 32);
        bad |= a + 1 < nc && cs[a + 1] < hi;
    }
    const uint64_t e = (a < nc && cs[a] == lo) ? a + 1 : a;   // first chunk start > lo
    if (e < nc && cs[e] <= hi) {
        w |= ((cs[e] - 1 - lo) << 12) | kCmEnd;
        bad |= e + 1 < nc && cs[e + 1] <= hi;
    }
    return w;
}

// A map of at most kCmLds chunks is searched in LDS: the block loads every chunk start in one
// round of parallel loads instead of a binary search's log2(nchunks) dependent ones (the kernel
// runs before every u16 pass, and a deep chain's late passes are made of such round trips).
constexpr uint32_t kCmLds = 1024;
__global__ __launch_bounds__(256) void chunk_map_kernel(PassParams p) {
    __shared__ uint64_t s_cs[kCmLds];
    const bool done = pass_done(p);      // (both loads in flight together)
    const uint64_t n = token_count(p);
    if (done) return;
    const uint64_t r = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (r < (n + kTileTok - 1) / kTileTok) p.status[r] = 0ull;
    if (p.cmap_next && r < (n + kWavePos - 1) / kWavePos) p.cmap_next[r] = 0ull;   // the scan ORs into it
    if (r == 0) { p.ctl[p.tick] = 0u; p.ctl[kCtlCover] = 0u; }   // this pass dirties the status words
    const uint64_t nc = p.nchunks;
    const bool in_lds = nc <= kCmLds;
    if ((uint64_t)blockIdx.x * 256u * kWavePos >= n) return;   // uniform: no range of this block is live
    if (in_lds) {
        for (uint32_t i = threadIdx.x; i < nc; i += 256u) s_cs[i] = p.cstart[i];
        __syncthreads();
    }
    const uint64_t lo = r * kWavePos, hi = lo + kWavePos;
    if (lo >= n) return;
    bool bad = false;
    const uint64_t w = in_lds ? cm_word(s_cs, nc, lo, hi, bad) : cm_word(p.cstart, nc, lo, hi, bad);
    if (bad) flag_error(p.ctl, KARG(sticky), 16u);   // chunks shorter than a wave range: host bug
    p.cmap[r] = w;
}

// Tokens of tile Tn into x (the same straight-line loads as load_tile; near the buffer end the
// lanes' tokens again one by one), and the wave ranges' chunk-map words, packed in one register:
// lane l holds dword l & 1 of sub-tile (l >> 1) & 1's word (read back with v_readlane where used;
// a wave-uniform value in a VGPR of its own per dword was 8 registers the kernel does not have).
// Sub-tile j of wave w: tokens [j kSubTok + 1024 w, +1024), wave range Tn kGroupsTok + j kWaves + w.
__device__ __forceinline__ void load_tok(const PassParams& p, uint64_t n, uint32_t Tn, uint32_t wave, int lane,
                                         uint32_t (&x)[kSt][8], uint32_t (&nxt)[kSt], uint32_t& cw) {
    const uint8_t* in = reinterpret_cast<const uint8_t*>(p.in);
    const uint64_t tile0 = (uint64_t)Tn * kTileTok;
    const uint64_t left = n > tile0 ? n - tile0 : 0;
    const __amdgpu_buffer_rsrc_t rd = rsrc_at(in + 2 * tile0, (2 * left) & ~3ull);
    const uint64_t r0 = (uint64_t)Tn * kGroupsTok, nr = (n + kWavePos - 1) / kWavePos;
    const __amdgpu_buffer_rsrc_t rm = rsrc_at(p.cmap + r0, nr > r0 ? 8 * (nr - r0) : 0);
#pragma unroll
    for (int j = 0; j < kSt; ++j) {
        const uint32_t wrel = (uint32_t)j * kSubTok + wave * kWavePos;
        const int o = 2 * (int)(wrel + 16u * (uint32_t)lane);
        const auto v0 = __builtin_amdgcn_raw_buffer_load_b128(rd, o, 0, kLdPol);
        const auto v1 = __builtin_amdgcn_raw_buffer_load_b128(rd, o + 16, 0, kLdPol);
        x[j][0] = v0[0]; x[j][1] = v0[1]; x[j][2] = v0[2]; x[j][3] = v0[3];
        x[j][4] = v1[0]; x[j][5] = v1[1]; x[j][6] = v1[2]; x[j][7] = v1[3];
        nxt[j] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rd, (int)(2 * (wrel + kWavePos)), 0, 0);
    }
    static_assert(kSt == 2, "chunk-map words: 4 dwords per wave");
    const uint32_t cl = (lane16_here() >> 4) & 3u;
    cw = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rm, (int)(8u * ((cl >> 1) * (uint32_t)kWaves + wave) + 4u * (cl & 1u)), 0, 0);
    const uint32_t rn = (uint32_t)(left > 0x7FFFFFFFull ? 0x7FFFFFFFull : left);
#pragma unroll
    for (int j = 0; j < kSt; ++j) {
        const uint32_t wrel = (uint32_t)j * kSubTok + wave * kWavePos;
        if (rn > wrel && rn - wrel < kWavePos + 16u) {   // uniform: the buffer end is near this range
            const __amdgpu_buffer_rsrc_t r = rsrc_at(in + 2 * tile0, 2 * left);
            const int o = 2 * (int)(wrel + 16u * (uint32_t)lane);
            nxt[j] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, (int)(2 * (wrel + kWavePos)), 0, 0);
#pragma unroll
            for (int q = 0; q < 8; ++q)
                x[j][q] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, o + 4 * q, 0, 0) |
                          ((uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, o + 4 * q + 2, 0, 0) << 16);
        }
    }
}

// Lookup of one pair key in the token table.  kHash: 0 the 2-choice table in global memory (L2),
// 1 the 2-choice table in LDS (byte address tab), 2 a one-probe table in LDS (small maps: the host
// found a multiplier that puts every key in its own bucket).
template <int kHash>
__device__ __forceinline__ uint32_t tok_get(const PassParams& p, uint32_t tab, uint32_t key) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    typedef __attribute__((address_space(3))) u32x2 lds_u32x2;
    const uint32_t b1 = bucket_hash(key, p.hmul1, p.hshift);
    if constexpr (kHash == 2) {
        const u32x2 x = *(const lds_u32x2*)(uintptr_t)(tab + 8u * b1);
        return x[0] == key ? x[1] : 0u;
    }
    const uint32_t b2 = bucket_hash(key, p.hmul2, p.hshift);
    u32x2 x, y;
    if constexpr (kHash == 1) {
        x = *(const lds_u32x2*)(uintptr_t)(tab + 8u * b1);
        y = *(const lds_u32x2*)(uintptr_t)(tab + 8u * b2);
    } else {
        const u32x2* g = reinterpret_cast<const u32x2*>(p.hbuckets);
        x = g[b1];
        y = g[b2];
    }
    return (x[0] == key ? x[1] : 0u) | (y[0] == key ? y[1] : 0u);
}

// Phase 1 of one wave range of tokens (sub-tile j): 16 lookups per lane, the output token of each
// position if it lands (merged value or the token itself, big-endian, two per register), buffer
// and chunk ends; returns the lane's merge mask, sets live when a surviving merge's value is a key
// component (value word bit 30: a pass with no such merge leaves no mergeable pair behind, see
// scan_tokens_kernel).  rem: tokens from the range start to the buffer end; cwl: low word of the
// range's chunk-map word.
// next_ok (fused passes): the token after position rem - 1 is valid (it is the next wave range's
// first token, staged at position rem), so position rem - 1 may merge with it.
template <int kHash>
__device__ __forceinline__ uint32_t phase1_tok(const PassParams& p, uint32_t tab, const uint32_t (&x)[8],
                                               uint32_t nxt, uint32_t rem, uint32_t cwl, int lane, int j,
                                               TileStateT<kSt>& st, uint32_t& live, bool next_ok = false) {
    // next lane's first token (wave_shl:1); lane 63 keeps the token after the wave's range
    const uint32_t nbw = (uint32_t)__builtin_amdgcn_update_dpp((int)nxt, (int)x[0], 0x130, 0xF, 0xF, false);
    uint32_t r[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int h = k >> 1;
        const uint32_t key = (k & 1) ? __builtin_amdgcn_alignbyte(h < 7 ? x[h + 1] : nbw, x[h], 2) : x[h];
        r[k] = tok_get<kHash>(p, tab, key);
    }
    uint32_t racc = 0;
#pragma unroll
    for (int k = 0; k < 16; k += 2) racc |= r[k] | r[k + 1];
    uint32_t lv = (racc >> 30) & 1u;
    uint32_t m32 = 0;   // even positions in bits 0..14, odd positions in bits 16..30
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        const uint32_t R = __builtin_amdgcn_perm(r[2 * h + 1], r[2 * h], 0x05040100u);     // both values
        const uint32_t hit = __builtin_amdgcn_perm(r[2 * h + 1], r[2 * h], 0x0B0B0909u);   // bit 31 -> half
        st.v[j][h] = (hit & R) | (~hit & x[h]);
        m32 |= (hit & 0x00010001u) << (2 * h);
    }
    uint32_t m = (m32 & 0xFFFFu) | (m32 >> 15);
    const bool has_end = (cwl & kCmEnd) != 0u;
    if (rem <= kWavePos || has_end) {   // uniform; rare
        const uint32_t l16 = lane16_here();   // (not a hoisted per-lane constant: see lane16_here)
        const int32_t rr = (int32_t)(rem > 2u * kWavePos ? 2u * kWavePos : rem) - (int32_t)l16;
        const uint32_t vmask = rr >= 16 ? 0xFFFFu : (rr <= 0 ? 0u : ((1u << rr) - 1u));
        uint32_t mm = m & (next_ok ? vmask : ((vmask >> 1) | (rr > 16 ? 0x8000u : 0u)));
        uint32_t forced = (!next_ok && rr >= 1 && rr <= 16) ? (1u << (rr - 1)) : 0u;   // the buffer's last token
        if (has_end) {                                                     // a chunk's last token
            const uint32_t e = ((cwl >> 12) & 0x7FFu) - l16;
            if (e < 16u) { mm &= ~(1u << e); forced |= 1u << e; }
        }
        if (__ballot(forced != 0)) {   // a cut merge emits its own token
#pragma unroll
            for (int h = 0; h < 8; ++h) {
                const uint32_t fm = (((forced >> (2 * h)) & 1u) ? 0x0000FFFFu : 0u) |
                                    (((forced >> (2 * h + 1)) & 1u) ? 0xFFFF0000u : 0u);
                st.v[j][h] = (st.v[j][h] & ~fm) | (x[h] & fm);
            }
        }
        m = mm;
        st.mv[j] = mm | (vmask << 16);
        // only the merges that survive the buffer and chunk ends count (their lookups, still live:
        // a second lookup here, sixteen results in flight, made the kernel spill)
        uint32_t lacc = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) lacc |= ((mm >> k) & 1u) ? r[k] : 0u;
        lv = (lacc >> 30) & 1u;
    } else {
        st.mv[j] = m | 0xFFFF0000u;
    }
    live |= lv;
    return m;
}

// Emission of sub-tile j's wave range (as emit_tile), its chunk start from the chunk-map word.
// rem: tokens from the range start to the buffer end; wtok: the range's first input token.
__device__ __forceinline__ void emit_tok(const PassParams& p, uint64_t wtok, uint32_t rem, uint32_t cwl, uint32_t cwh,
                                         int, int j, const TileStateT<kSt>& st, const uint32_t* gin,
                                         uint32_t C, uint64_t O, uint8_t* stg, uint32_t wave, bool has_coff,
                                         bool inplace = true) {
    // the lane index computed here (inline asm is never hoisted): the copy-out's per-lane offsets,
    // hoisted out of the loop as constants, were spilled, and each reload's vmcnt wait made the
    // emission wait for the next tile's loads
    const int lane = (int)(lane16_here() >> 4);
    uint8_t* out = reinterpret_cast<uint8_t*>(p.out);
    const uint64_t obase = (2ull * O) & ~15ull;
    const uint32_t orel = (uint32_t)(2ull * O - obase);
    const __amdgpu_buffer_rsrc_t ro = rsrc_at(out + obase, p.out_cap > obase ? p.out_cap - obase : 0);
    const uint32_t cg = uni(gin[C]);
    const uint32_t goff = uni(gin[2 + C]);   // tokens before this wave range in the tile
    const uint32_t gb = orel + 2u * goff;    // output byte of the wave range, from obase
    const bool cstart = has_coff && (cwl & kCmStart) != 0u;
    if (__ballot(st.mv[j] != 0xFFFFFFFFu) == 0) {
        // dense: every pair merges, so the only possible chunk start is the range's first token
        if (cstart && lane == 0) {
            KARG(chunk_off)[cwh] = O + goff;
            if (inplace && p.cmap_next) cm_mark(p, p.cmap_next, O + goff, cwh);
        }
        emit_dense(st.v[j], cg, gb - (gb & ~15u), ro, gb & ~15u, lane);
        return;
    }
    const uint32_t m = st.mv[j] & 0xFFFFu, vmask = st.mv[j] >> 16;
    const uint32_t c = __builtin_amdgcn_ubfe(st.ex[j], 16u * cg + 15u, 1);
    const uint32_t lane_off = __builtin_amdgcn_ubfe(st.ex[j], 16u * cg, 15);
    const uint32_t mc = c ? m : (m & ~1u);
    const uint32_t sst = mc & ~(mc << 1);
    const uint32_t rodd = mc & ~(mc + (sst & 0xAAAAu));
    const uint32_t M = (mc & ~rodd & 0x5555u) | (rodd & 0xAAAAu);
    const uint32_t L = ~((M << 1) | (c ^ 1u)) & vmask;
    if (cstart) {
        const uint32_t e = (cwl & 0x7FFu) - lane16_here();
        if (e < 16u) {
            const uint64_t P = O + goff + lane_off + __popc(L & ((1u << e) - 1u));
            KARG(chunk_off)[cwh] = P;
            if (inplace && p.cmap_next) cm_mark(p, p.cmap_next, P, cwh);
        }
    }
    const uint32_t wcnt = uni(lane_u32(lane_off + __popc(L), 63));
    // in place: output = input when nothing merged before this range or in it
    if (inplace && wcnt == (rem < kWavePos ? rem : kWavePos) && O + goff == wtok) return;
    // one part: the stage holds the range's at most 1024 tokens
    const uint32_t x0 = wave * (uint32_t)kStageTok;   // the wave's stage, logical bytes
    stage_b16_pad(st.v[j], L, stg, x0 + (gb & 15u) + 2u * lane_off);
    const CopyPart cp = {gb & ~15u, gb & 15u, (gb & 15u) + 2u * wcnt};
    CopyData<kCopyBlkTok> d;
    copy_read_pad(stg, x0, cp, lane, d);
    copy_store<kCopyBlkTok, false>(ro, cp, lane, d);   // (branch-free here: f2 +2.5 %)
}

// ===========================================================================================
// Passes 1 and 2 of a general map in one kernel (kFused): the u16 scan kernel with a front end that
// runs the first pass on each wave range's 1024 bytes.  The first pass restarts after every byte
// pair it does not merge (L[i + 1] = 1 when m[i] = 0), so a wave range's carry-in (does its first
// byte land) follows from the 64 bytes before it: the last restart there lands, and the positions
// after it alternate while every pair merges (tools/halo_model.py checks the rule against whole
// passes).  The range's first-pass tokens go through the wave's stage into 16 tokens per lane,
// followed by the next range's first token; from there the second pass is the u16 scan as it is
// (its carries and all offsets through the look-back).  The intermediate tokens never leave LDS.
// A range whose halo holds no restart (a run of merging pairs longer than the halo) sets
// *p.fused_fail and the done word, and the host runs the two-kernel chain instead.
// ===========================================================================================
constexpr uint32_t kHalo = 64;   // bytes before a wave range, one per lane

// Bytes 2h and 2h + 1 of word xw (h & 1 picks the word's half) as two big-endian u16 tokens.
__device__ __forceinline__ uint32_t be_pair(uint32_t xw, int h) {
    return __builtin_amdgcn_perm(xw, xw, (h & 1) ? 0x030C020Cu : 0x010C000Cu);
}

// Lane function of one wave range (lane_wave_fns' first part): the exclusive prefix word under
// both wave carry-in hypotheses, no wave-function record.
__device__ __forceinline__ uint32_t lane_ex1(uint32_t m, uint32_t vm) {
    const uint64_t nonid = __ballot(m != 0xFFFFu);
    const uint32_t mc = (m & ~1u) | (m << 16);
    const uint32_t sst = mc & ~pk_shl1(mc);
    const uint32_t rodd = mc & ~pk_add(mc, sst & 0xAAAAAAAAu);
    const uint32_t M = (mc & ~rodd & 0x55555555u) | (rodd & 0xAAAAAAAAu);
    const uint32_t L = ~(pk_shl1(M) | 1u) & (vm | (vm << 16));
    const uint32_t cnt0 = __popc(L & 0xFFFFu), cnt1 = __popc(L >> 16);
    const uint64_t cmask = __ballot(((M >> 31) & 1u) == 0u);
    const uint64_t D = cmask & nonid, Mi = ~nonid, A = D << 1;
    const uint64_t Y = ((Mi + A) ^ Mi ^ A) | A;
    const uint64_t F = nonid ? ((nonid & (0ull - nonid)) << 1) - 1ull : ~0ull;
    const uint64_t CI0 = Y, CI1 = Y | F;
    const uint32_t packed = lane_sel(CI0, cnt0, cnt1) | (lane_sel(CI1, cnt0, cnt1) << 16);
    const uint32_t incl = wave_scan(packed);
    return (incl - packed) | lane_sel(CI0, 0u, 0x8000u) | lane_sel(CI1, 0u, 0x80000000u);
}

// A lane's landing mask L, merge starts M and token offset under wave carry-in C (1: the range's
// first position lands), as emit_tok derives them.
__device__ __forceinline__ void lands1(uint32_t m, uint32_t vmask, uint32_t ex, uint32_t C, uint32_t& L,
                                       uint32_t& M, uint32_t& off) {
    const uint32_t c = __builtin_amdgcn_ubfe(ex, 16u * C + 15u, 1);
    off = __builtin_amdgcn_ubfe(ex, 16u * C, 15);
    const uint32_t mc = c ? m : (m & ~1u);
    const uint32_t sst = mc & ~(mc << 1);
    const uint32_t rodd = mc & ~(mc + (sst & 0xAAAAu));
    M = (mc & ~rodd & 0x5555u) | (rodd & 0xAAAAu);
    L = ~((M << 1) | (c ^ 1u)) & vmask;
}

// Bytes of tile Tn for the fused kernel: a lane's 16 bytes (x[j][0..3]), its halo byte (x[j][4]:
// byte wb - 64 + lane of its wave range wb) and the 4 bytes after the range (nxt[j]); exact byte
// loads near the buffer end (as load_tile).
__device__ __forceinline__ void load_fused(const PassParams& p, uint64_t n, uint32_t Tn, uint32_t wave, int lane,
                                           uint32_t (&x)[kSt][8], uint32_t (&nxt)[kSt]) {
    const uint8_t* in = reinterpret_cast<const uint8_t*>(p.in);
    const uint64_t tile0 = (uint64_t)Tn * kTileTok;
    const uint64_t left = n > tile0 ? n - tile0 : 0;
    const __amdgpu_buffer_rsrc_t rd = rsrc_at(in + tile0, left & ~3ull);
#pragma unroll
    for (int j = 0; j < kSt; ++j) {
        const uint32_t wrel = (uint32_t)j * kSubTok + wave * kWavePos;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rd, (int)(wrel + 16u * (uint32_t)lane), 0, kLdPol);
        x[j][0] = v[0]; x[j][1] = v[1]; x[j][2] = v[2]; x[j][3] = v[3];
        nxt[j] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rd, (int)(wrel + kWavePos), 0, 0);
        const uint64_t wb = tile0 + wrel;
        x[j][4] = 0u;
        // (uniform) only a range that holds bytes reads its halo.  Round 5's intermittent illegal
        // memory access: this load had no `wb < n` test, so the last tile's empty ranges read 64
        // bytes up to ~32 KiB past the input; with an input allocation of exactly up16(n) bytes (a
        // pooled context regrown for n) that ran into unmapped pages.
        if (wb >= kHalo && wb < n)
            x[j][4] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc_at(in + wb - kHalo, kHalo), lane, 0, 0);
    }
    const uint32_t rn = (uint32_t)(left > 0x7FFFFFFFull ? 0x7FFFFFFFull : left);
#pragma unroll
    for (int j = 0; j < kSt; ++j) {
        const uint32_t wrel = (uint32_t)j * kSubTok + wave * kWavePos;
        if (rn > wrel && rn - wrel < kWavePos + 16u) {   // uniform: the buffer end is near this range
            const __amdgpu_buffer_rsrc_t r = rsrc_at(in + tile0, left);
            uint32_t nw = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                nw |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)(wrel + kWavePos) + b, 0, 0) << (8 * b);
            nxt[j] = nw;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t d = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    d |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)(wrel + 16u * (uint32_t)lane) + 4 * q + b, 0, 0)
                         << (8 * b);
                x[j][q] = d;
            }
        }
    }
}

// Front end of one wave range [wb, wb + 1024) of bytes: the first pass, its tokens compacted
// through the wave's stage into x (16 per lane) with the next range's first token after them, and
// the second pass's inputs: nxt (that token), rem2 (tokens of the range; 2048 when it holds 1024
// and the next token is valid), next_ok, and the range's chunk-map word (cwl, cwh) in token
// positions.  Wave-uniform control throughout.
template <int kHash>
__device__ __forceinline__ void fused_front(const PassParams& p, uint32_t tab, uint32_t (&x)[8], uint32_t& nxt,
                                            uint64_t wb, uint64_t n, int lane, uint32_t wave, uint8_t* stg,
                                            uint32_t& rem2, bool& next_ok, uint32_t& cwl, uint32_t& cwh, uint32_t& C2) {
    const uint32_t hb = x[4] & 0xFFu;
    const uint32_t nb4 = nxt;
    const uint64_t left = n > wb ? n - wb : 0;
    const uint32_t rem1 = (uint32_t)(left > 2u * kWavePos ? 2u * kWavePos : left);
    // chunk geometry: wb = q cs + r; the first chunk start at or after wb is s bytes on
    const uint64_t cs = p.cs;
    uint64_t q = __umul64hi(wb, p.cs_magic);
    uint64_t r = wb - q * cs;
    if (r >= cs) { q += 1; r -= cs; }
    if (r >= cs) { q += 1; r -= cs; }
    const uint64_t s = r ? cs - r : 0;
    uint32_t cwl1 = 0;
    if (s < kWavePos) cwl1 |= kCmStart | (uint32_t)s;
    if (r && s >= 1 && s <= kWavePos) cwl1 |= kCmEnd | ((uint32_t)(s - 1) << 12);

    // first pass over the range's bytes as big-endian tokens
    uint32_t t[8];
#pragma unroll
    for (int h = 0; h < 8; ++h) t[h] = be_pair(x[h >> 1], h);
    TileStateT<kSt> s1;
    uint32_t live1 = 0;
    const uint32_t m1 = phase1_tok<kHash>(p, tab, t, (nb4 & 0xFFu) << 8, rem1, cwl1, lane, 0, s1, live1);
    const uint32_t vm1 = s1.mv[0] >> 16;
    const uint32_t ex1 = lane_ex1(m1, vm1);

    // Carries from the halo (lane l: byte wb - 64 + l).  Pass 1: the last restart (a byte whose
    // left pair does not merge, or a chunk start) lands and the merging pairs after it alternate, so
    // C1 = 1 unless byte wb - 1 lands and merges with byte wb.  Pass 2 the same way over the halo's
    // first-pass tokens after its first restart, up to the range's first token: C2 = 1 unless the
    // halo's last first-pass token lands in pass 2 and merges with it.  A halo with no restart for
    // either pass cannot resolve the range.
    uint32_t C1 = 1u;
    C2 = 1u;
    if (wb != 0 && r != 0 && left != 0) {
        const uint32_t b0 = uni(lane_u32(x[0], 0)) & 0xFFu;   // byte wb: lane 63's right neighbour
        const uint32_t hn = (uint32_t)__builtin_amdgcn_update_dpp((int)b0, (int)hb, 0x130, 0xF, 0xF, false);
        const int cl = r <= kHalo ? (int)kHalo - (int)r : -1;   // a chunk start in the halo, at lane cl
        const uint32_t v1 = lane + 1 != cl ? tok_get<kHash>(p, tab, (hb << 8) | (hn << 24)) : 0u;
        const bool hit = (v1 >> 31) != 0u;
        const uint64_t hm = __ballot(hit);
        const uint64_t below = (2ull << lane) - 1ull;   // lanes 0..lane (lane 63: all)
        const bool rst = lane == cl || (lane >= 1 && ((hm >> (lane - 1)) & 1ull) == 0ull);
        const uint64_t R = __ballot(rst);
        bool ok = R != 0;
        if (ok) {
            const int lr = 63 - __clzll(R);
            C1 = (((63 - lr) & 1) == 0 && ((hm >> 63) & 1ull)) ? 0u : 1u;
            // first-pass landings from the first restart on, and their tokens
            const int r0 = __builtin_ctzll(R);
            const uint64_t rl = R & below;
            const bool land = lane >= r0 && rl != 0 && ((lane - (63 - __clzll(rl))) & 1) == 0;
            const uint64_t LM = __ballot(land);
            const uint32_t t1 = hit ? (v1 & 0xFFFFu) : (hb << 8);
            const uint32_t tf = uni(lane_u32(C1 ? (s1.v[0][0] & 0xFFFFu) : (s1.v[0][0] >> 16), 0));   // range's first token
            const int nl = lane + 1 + (hit ? 1 : 0);   // next landing (for a landing lane)
            uint32_t tn = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * (nl < 64 ? nl : 63), (int)t1);
            if (nl >= 64) tn = tf;
            const uint32_t v2 = (land && nl != cl) ? tok_get<kHash>(p, tab, t1 | (tn << 16)) : 0u;
            const uint64_t H2 = __ballot((v2 >> 31) != 0u);
            const uint64_t lprev = LM & (below >> 1);   // landings below this lane
            const bool rst2 = land && (lane == cl || (lprev != 0 && ((H2 >> (63 - __clzll(lprev))) & 1ull) == 0ull));
            const uint64_t R2 = __ballot(rst2);
            ok = R2 != 0;
            if (ok) {
                const int lr2 = 63 - __clzll(R2), lst = 63 - __clzll(LM);   // last restart, last landing
                const uint64_t span = (lst == 63 ? ~0ull : ((2ull << lst) - 1ull)) & ~((1ull << lr2) - 1ull);
                const bool l2 = ((__popcll(LM & span) - 1) & 1) == 0;   // the last landing lands in pass 2
                C2 = (l2 && ((H2 >> lst) & 1ull)) ? 0u : 1u;
            }
        }
        // A chunk start at byte wb + 1 whose byte wb merged into the halo's last token (C1 = 0) is the
        // range's first first-pass token: the pair before it is cut in pass 2 as well, so it lands.
        // (Round 6: the halo's pass-2 rule saw the pair as mergeable and gave C2 = 0; the range's
        // count then disagreed with the carry the tile resolve gave its emission, and the next
        // range's tokens overwrote its last one, in whichever order the waves stored.)
        if (s == 1u && C1 == 0u) C2 = 1u;
        if (!ok) {   // no restart: this kernel cannot resolve the range (the host falls back)
            if (lane == 0) {
                *KARG(fused_fail) = 1u;
                if (uint32_t* dn = KARG(done)) *dn = p.pass_id;
                // fail fast: every later ticket claim gets a tile past the end, so the workgroups
                // finish the tiles they hold (all of whose predecessors are claimed) and leave
                atomicMax(KARG(ctl), 0x80000000u);
            }
        }
    }
    uint32_t L1, M1, off1;
    lands1(m1, vm1, ex1, C1, L1, M1, off1);
    const uint32_t c1 = uni(lane_u32(off1 + __popc(L1), 63));

    // the next range's first token (the first landing at or after wb + 1024)
    const uint32_t Cn = (uni(lane_u32(M1, 63)) >> 15) & 1u;   // 1: byte wb + 1024 merged into our last token
    const uint64_t fnx = wb + kWavePos + Cn;
    next_ok = fnx < n && !(r != 0 && s == (uint64_t)kWavePos + Cn);
    uint32_t tokn = 0;
    if (next_ok) {
        const uint32_t a = (nb4 >> (8 * Cn)) & 0xFFu, b = (nb4 >> (8 * (Cn + 1))) & 0xFFu;
        const bool pv = fnx + 1 < n && !(r != 0 && s == (uint64_t)kWavePos + Cn + 1);
        const uint32_t v = pv ? tok_get<kHash>(p, tab, (a << 8) | (b << 24)) : 0u;
        tokn = (v >> 31) ? (v & 0xFFFFu) : (a << 8);
    }

    // compaction through the stage, the next token after the range's tokens, 16 tokens per lane back
    const uint32_t x0 = wave * (uint32_t)kStageTok;
    stage_b16_pad(s1.v[0], L1, stg, x0 + 2u * off1);
    if (next_ok && lane == 0) *reinterpret_cast<uint16_t*>(stg + stage_phys(x0 + 2u * c1)) = (uint16_t)tokn;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint2 d = *reinterpret_cast<const uint2*>(stg + stage_phys(x0 + 32u * (uint32_t)lane + 8u * k));
        x[2 * k] = d.x;
        x[2 * k + 1] = d.y;
    }
    nxt = tokn;
    rem2 = (c1 == kWavePos && next_ok) ? 2u * kWavePos : c1;

    // chunk start of this range in token positions (it lands: the pair before it is cut)
    cwl = 0u;
    cwh = 0u;
    if (s < kWavePos && s < left) {
        const uint32_t sl = (uint32_t)s >> 4, sb = (uint32_t)s & 15u;
        const uint32_t te = uni(__builtin_amdgcn_readlane((int)(off1 + __popc(L1 & ((1u << sb) - 1u))), (int)sl));
        cwl = kCmStart | te;
        if (s != 0 && te != 0) cwl |= kCmEnd | ((te - 1u) << 12);
        cwh = (uint32_t)(r ? q + 1 : q);
    }
}

template <int kHash, bool kFused = false>
__global__ __launch_bounds__(kThreads) void scan_tokens_kernel(PassParams p) {
    constexpr bool kHashLds = kHash != 0;
    extern __shared__ __attribute__((aligned(16))) uint2 s_tokhash[];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[kWaves * kStageTokPhys];   // padded
    
    __shared__ __attribute__((aligned(16))) uint32_t s_wfn[kRing][kGroupsTok][4];
    __shared__ uint32_t s_gin[kRing][kGroupsTok][4];
    __shared__ uint32_t s_tfn[kRing][4];
    __shared__ uint64_t s_O[kRing];
    __shared__ uint32_t s_C[kRing];
    __shared__ uint32_t s_tk[kRing];
    __shared__ uint32_t s_p1cnt[kRing];
    __shared__ uint32_t s_rdone, s_lbdone, s_tkdone;

    // an earlier pass merged nothing (uniform over the grid); both loads in flight together
    const bool done = !kFused && pass_done(p);
    const uint64_t n = kFused ? p.n : uni64(token_count(p));   // fused: bytes
    if (done) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t wave = uni((uint32_t)tid >> 6);
    const bool has_coff = p.chunk_off != nullptr;
    const uint32_t ntiles = (uint32_t)((n + kTileTok - 1) / kTileTok);
    // the grid was sized for the token bound; workgroups past the tiles the previous pass left leave
    // before copying the table (the ones below claim every ticket)
    if (blockIdx.x >= ntiles) return;
    // tokens from sub-tile j's wave range start of tile T to the buffer end (clamped)
    auto rem_of = [&](uint32_t T, int j) {
        const uint64_t w0 = (uint64_t)T * kTileTok + (uint64_t)j * kSubTok + wave * kWavePos;
        const uint64_t l = n > w0 ? n - w0 : 0;
        return (uint32_t)(l > 0x7FFFFFFFull ? 0x7FFFFFFFull : l);
    };

    if constexpr (kHashLds) {
        // LDS-DMA, all loads in flight (the LDS region is rounded up to whole KiB: a wave-
        // instruction fills 1 KiB; the lanes past the table load its last unit again)
        const uint4* src = reinterpret_cast<const uint4*>(p.hbuckets);
        uint4* dst = reinterpret_cast<uint4*>(s_tokhash);
        const uint32_t nu = p.hbytes / 16u;
#pragma unroll
        for (uint32_t k = 0; k < kHashLdsMax / 16u / kThreads; ++k) {
            const uint32_t u0 = wave * 64u + k * kThreads;   // uniform
            if (u0 < nu)
                __builtin_amdgcn_global_load_lds(
                    (__attribute__((address_space(1))) void*)(src + (u0 + lane < nu ? u0 + lane : nu - 1)),
                    (__attribute__((address_space(3))) void*)(dst + u0), 16, 0, 0);
        }
    }
    if constexpr (!kFused) {
        // Chained u16 passes (round 6): the next pass's status words and ticket word (the other of
        // two sets; the previous pass used them) and the map the pass after next builds (the one the
        // previous pass read) are zeroed here over the live workgroups; this pass's own were zeroed by
        // the previous pass, or by chunk_map_kernel before the first.  No count-out at the end: the
        // next pass needs nothing from this one's tail.
        // These stores run beside this pass's ticket atomics and status publishes, some on the same
        // cache lines (the control block and the first status words share one): agent-scope
        // stores, coherent with them, not plain stores into an XCD's L2.
        const uint64_t live = gridDim.x < ntiles ? gridDim.x : ntiles;
        if (p.cmap_zero) {
            const uint64_t nr = (n + kWavePos - 1) / kWavePos;
            for (uint64_t i = (uint64_t)blockIdx.x * kThreads + tid; i < nr; i += live * kThreads)
                __hip_atomic_store(p.cmap_zero + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (p.status_zero)
            for (uint64_t i = (uint64_t)blockIdx.x * kThreads + tid; i < ntiles; i += live * kThreads)
                __hip_atomic_store(p.status_zero + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (blockIdx.x == 0 && tid == 0) {
            if (p.status_zero) __hip_atomic_store(p.ctl + (p.tick ^ kCtlTickAlt), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(p.ctl + kCtlCover, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // status words dirtied
        }
    }
    if (tid == 0) {
        s_tk[kRing - 2] = atomicAdd(p.ctl + p.tick, 1u);   // T
        s_tk[kRing - 1] = atomicAdd(p.ctl + p.tick, 1u);   // Tq, the tile after it
        for (int r = 0; r < kRing; ++r) s_p1cnt[r] = 0;
        s_rdone = 0; s_lbdone = 0; s_tkdone = 0;
    }
    __syncthreads();
    const uint32_t tab = kHashLds ? uni(lds_addr(s_tokhash)) : 0u;
    uint32_t T = uni(s_tk[kRing - 2]);
    uint32_t Tp = kNone;
    uint32_t Tq = uni(s_tk[kRing - 1]);
    if (T >= ntiles || Tq >= ntiles) Tq = kNone;
    __syncthreads();
    uint32_t it = 0;

    {
        uint32_t xa[kSt][8], xb[kSt][8], na[kSt], nb[kSt], ca = 0u, cb = 0u;
#pragma unroll
        for (int j = 0; j < kSt; ++j) na[j] = nb[j] = 0u;
        
        if (T < ntiles) {
            if constexpr (kFused) load_fused(p, n, T, wave, lane, xa, na);
            else load_tok(p, n, T, wave, lane, xa, na, ca);
        }
        TileStateT<kSt> sa, sb;
        uint64_t lbs[kLbWin];
        uint32_t cwp = 0u;   // Tp's chunk-map words, packed as load_tok packs them
        auto step = [&](uint32_t (&x)[kSt][8], uint32_t (&nxt)[kSt], uint32_t& cw, uint32_t (&xq)[kSt][8],
                        uint32_t (&nxtq)[kSt], uint32_t& cwq, TileStateT<kSt>& sc, const TileStateT<kSt>& sp) {
            const uint32_t slot = it & (kRing - 1), pslot = (it - 1) & (kRing - 1);
            // the lane index per iteration (inline asm is never hoisted): per-lane constants derived
            // from it and hoisted out of the loop took the registers this kernel spilled (19-23 VGPRs
            // at one point), and each reload's vmcnt wait held its phase for the next tile's loads
            const int lane = (int)(lane16_here() >> 4);
            uint64_t stamp[7];
            const bool stamping = kTiming && p.debug != nullptr;
            if (stamping) stamp[0] = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): T's tokens and map words have landed
            if (stamping) stamp[1] = __builtin_amdgcn_s_memtime();

            uint32_t cwl[kSt], cwh[kSt];
#pragma unroll
            for (int j = 0; j < kSt; ++j) {
                cwl[j] = kFused ? 0u : lane_u32(cw, 2 * j);   // fused: from the front end
                cwh[j] = kFused ? 0u : lane_u32(cw, 2 * j + 1);
            }
            if (Tq < ntiles) {
                if constexpr (kFused) load_fused(p, n, Tq, wave, lane, xq, nxtq);
                else load_tok(p, n, Tq, wave, lane, xq, nxtq, cwq);
            }
            uint32_t tk = kNone;
            if (tid == kTkTid && Tq < ntiles) tk = atomicAdd(p.ctl + KARG(tick), 1u);
            asm volatile("" ::: "memory");

            bool lbw = wave == 0;
            if (T < ntiles) {
                if (wave >= (uint32_t)kPrioP1Wave) __builtin_amdgcn_s_setprio(kPrioP1);
                uint32_t m[kSt], live = 0;
                uint32_t rem2[kSt], C2[kSt];
                bool nok[kSt];
                if constexpr (kFused) {
#pragma unroll
                    for (int j = 0; j < kSt; ++j)
                        fused_front<kHash>(p, tab, x[j], nxt[j], (uint64_t)T * kTileTok + (uint64_t)j * kSubTok + wave * kWavePos,
                                           n, lane, wave, s_stage, rem2[j], nok[j], cwl[j], cwh[j], C2[j]);
#pragma unroll
                    for (int j = 0; j < kSt; ++j)
                        m[j] = phase1_tok<kHash>(p, tab, x[j], nxt[j], rem2[j], cwl[j], lane, j, sc, live, nok[j]);
                } else {
#pragma unroll
                    for (int j = 0; j < kSt; ++j)
                        m[j] = phase1_tok<kHash>(p, tab, x[j], nxt[j], rem_of(T, j), cwl[j], lane, j, sc, live);
                }
                const uint32_t wl = __ballot(live) != 0 ? 1u : 0u;
                lane_wave_fns<kSt>(m, wave, lane, sc, s_wfn[slot], wl);
                if constexpr (kFused) {
                    // a fused range knows its carry-in (C2, from the halo): its wave function is the
                    // constant one, with the count under C2 and the carry into the next range (the
                    // range's tokens fill only its first rem2 positions, so the lane functions' own
                    // carry-out, past the unused positions, is not it)
#pragma unroll
                    for (int j = 0; j < kSt; ++j) {
                        uint32_t L2, M2, off2;
                        lands1(m[j], sc.mv[j] >> 16, sc.ex[j], C2[j], L2, M2, off2);
                        const uint32_t cnt = uni(lane_u32(off2 + __popc(L2), 63));
                        uint32_t co = 1u;
                        if (nok[j]) {
                            const uint32_t last = (rem2[j] > kWavePos ? kWavePos : rem2[j]) - 1u;
                            const uint32_t mb = uni(__builtin_amdgcn_readlane((int)M2, (int)(last >> 4)));
                            co = ((mb >> (last & 15u)) & 1u) ? 0u : 1u;
                        }
                        if (lane == 63) {
                            const uint32_t g = (uint32_t)j * kWaves + wave;
                            s_wfn[slot][g][0] = wl << 1;
                            s_wfn[slot][g][1] = co;
                            s_wfn[slot][g][2] = cnt;
                            s_wfn[slot][g][3] = cnt;
                        }
                    }
                }
                __builtin_amdgcn_s_setprio(0);
                uint32_t old = 0;
                if (lane == 0)
                    old = __hip_atomic_fetch_add(&s_p1cnt[slot], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
                old = uni(old);
                lbw = old == (uint32_t)kWaves * (it / kRing);
                if (old == (uint32_t)kWaves * (it / kRing + 1u) - 1u) {
                    resolve_tile<kGroupsTok, true, true>(p, T, lane, s_wfn[slot], s_gin[slot], s_tfn[slot]);
                    if (lane == 0) lds_release(&s_rdone, it + 1u);
                }
            }
            if (stamping) stamp[2] = __builtin_amdgcn_s_memtime();

            if (lbw && Tp < ntiles) {
                uint32_t C = 1u, how = 0xFFFFu, spins = 0, live = 0;
                uint64_t O = 0ull;
                const bool lb = Tp > 0;
                if (lb) lb_issue<true>(p, (int64_t)Tp - 1, lane, lbs);
                wait_ge(p, &s_rdone, it);
                const uint32_t tfl = uni(s_tfn[pslot][0]), tf1 = uni(s_tfn[pslot][1]);
                const uint32_t tf0 = tfl & 1u, tf2 = uni(s_tfn[pslot][2]), tf3 = uni(s_tfn[pslot][3]);
                if (lb) lb_finish<true>(p, Tp, lane, lbs, C, O, how, spins, live);
                live |= (tfl >> 1) & 1u;   // tiles up to and including Tp
                if (lane == 0) {
                    // (test hook: a broken tile count)
                    const uint64_t end = O + (C == 1u ? tf3 : tf2) + ((KARG(inject) & kInjectScanTok) ? kTileTok : 0u);
                    // a tile's tokens end within its own input (and the buffer): in place, a range
                    // past it would overwrite the next tile's unread input
                    const uint64_t in_end = (uint64_t)(Tp + 1u) * kTileTok < n ? (uint64_t)(Tp + 1u) * kTileTok : n;
                    if (C > 1u || O > (uint64_t)Tp * kTileTok || end > in_end) {
                        if (C <= 1u) record_error(p, 4u, Tp, 0xFFu, O, end, C);
                        O = 0; C = 2u;
                    }
                    s_C[pslot] = C;
                    s_O[pslot] = O;
                    lds_release(&s_lbdone, it + 1u);
                    const uint64_t fin = C > 1u ? 0ull : O + (C ? tf3 : tf2);
                    if (Tp > 0) st_publish(p.status + Tp, st_incl(C == 1u ? tf1 : tf0, fin) | (live ? kStLiveIncl : 0ull));
                    if (2ull * fin > p.out_cap) record_error(p, 2u, Tp, 0xFFu, O, fin, C);
                    if (Tp == ntiles - 1) {
                        // The fixpoint: this pass merged nothing, or none of its merges made a key
                        // component, so the next pass merges nothing (a pair of two tokens this pass
                        // left alone was looked up here and rejected; a new token is in no key).
                        const bool fixed = p.done && C <= 1u && (fin == n || !live);
                        *KARG(total) = fin;
                        if (uint64_t* co = KARG(chunk_off)) co[KARG(nchunks)] = fin;
                        if (fixed) *KARG(done) = KARG(pass_id);   // (reloaded: kept live, it was spilled)
                    }
                    if (kDebugRecord && p.debug) {
                        uint64_t* d = p.debug + 4ull * Tp;
                        d[0] = O;
                        d[1] = ((uint64_t)C << 32) | how;
                        d[2] = ((uint64_t)tf3 << 32) | tf2;
                        d[3] = ((uint64_t)tf1 << 32) | tf0;
                    }
                }
            }

            if (stamping) stamp[3] = __builtin_amdgcn_s_memtime();
            if (Tp < ntiles) {
                wait_ge(p, &s_lbdone, it + 1u);
                if (stamping) stamp[4] = __builtin_amdgcn_s_memtime();
                if (wave >= (uint32_t)kPrioEmWave) __builtin_amdgcn_s_setprio(kPrioEm);
                const uint32_t Cp = uni(s_C[pslot]);
                if (Cp <= 1u) {
                    const uint64_t Op = uni64(s_O[pslot]);
#pragma unroll
                    for (int j = 0; j < kSt; ++j) {
                        const uint64_t wtok = (uint64_t)Tp * kTileTok + (uint64_t)j * kSubTok + wave * kWavePos;
                        emit_tok(p, wtok, kFused ? 0u : rem_of(Tp, j), lane_u32(cwp, 2 * j), lane_u32(cwp, 2 * j + 1), lane, j, sp,
                                 s_gin[pslot][(uint32_t)j * kWaves + wave], Cp, Op, s_stage, wave, has_coff, !kFused);
                    }
                }
                __builtin_amdgcn_s_setprio(0);
            }
            if (stamping) stamp[5] = __builtin_amdgcn_s_memtime();
            if (tid == kTkTid) {
                s_tk[slot] = tk;
                lds_release(&s_tkdone, it + 1u);
            }
            uint32_t Tr = kNone;
            if (Tq < ntiles) {
                wait_ge(p, &s_tkdone, it + 1u);
                Tr = uni(s_tk[slot]);
                if (Tr >= ntiles) Tr = kNone;
            }
            if (stamping && Tp < ntiles && lane == 0) {
                stamp[6] = __builtin_amdgcn_s_memtime();
                uint64_t* w = p.debug + 8ull * ntiles + 8ull * ((uint64_t)Tp * kWaves + wave);
#pragma unroll
                for (int q = 0; q < 6; ++q) w[q] = stamp[q + 1] - stamp[q];
            }
            if constexpr (kFused) {   // (the front end's words, packed as load_tok packs them)
                const uint32_t cl = (lane16_here() >> 4) & 3u;
                cwp = cl == 0u ? cwl[0] : cl == 1u ? cwh[0] : cl == 2u ? cwl[1] : cwh[1];
            } else {
                cwp = cw;
            }
            Tp = T;
            T = Tq;
            Tq = Tr;
            ++it;
        };
        for (;;) {
            if (!(T < ntiles || Tp < ntiles)) break;
            step(xa, na, ca, xb, nb, cb, sa, sb);
            if (!(T < ntiles || Tp < ntiles)) break;
            step(xb, nb, cb, xa, na, ca, sb, sa);
        }
    }
}

}  // namespace seg

// Byte -> big-endian u16 (BasicTokenizationStrategy, tokenizer.rs:108-124).  A streaming copy
// that doubles the bytes: each thread loads one 8-byte input block and writes it as one 16-byte
// output block, so every store instruction of a wave covers 1 KiB of contiguous output, and the
// grid has one thread per block; the stores are non-temporal (1 GiB: 0.493 ms, 6.53 TB/s
// algorithmic = 82 % of HBM peak).
// Measured against it: 16-byte loads writing two 16-byte blocks each, 4 in flight per thread
// over 65,536 workgroups (0.607 ms); 8-byte blocks with 2 or 4 per thread, or fewer workgroups
// (0.55-0.62 ms).
// nt stores: 0.512-0.514 -> 0.492-0.494 ms per GiB (nt loads measured slower)
constexpr uint64_t kBasicMaxBlocks = 1u << 24;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
// bytes b0..b7 -> [0, b0, 0, b1, ..., 0, b7]
__device__ __forceinline__ v4u basic_expand8(v2u w) {
    v4u a;
    a[0] = __builtin_amdgcn_perm(w[0], 0u, 0x050C040Cu);
    a[1] = __builtin_amdgcn_perm(w[0], 0u, 0x070C060Cu);
    a[2] = __builtin_amdgcn_perm(w[1], 0u, 0x050C040Cu);
    a[3] = __builtin_amdgcn_perm(w[1], 0u, 0x070C060Cu);
    return a;
}
__global__ __launch_bounds__(256) void basic_expand_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                           uint8_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t n8 = n / 8;
    const v2u* src = reinterpret_cast<const v2u*>(in);
    v4u* dst = reinterpret_cast<v4u*>(out);
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < n8; i += stride) __builtin_nontemporal_store(basic_expand8(src[i]), dst + i);
    for (uint64_t k = n8 * 8 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        out[2 * k] = 0;
        out[2 * k + 1] = in[k];
    }
}

// End of a general map's chain enqueued without reading its pass count (the map's chain depth
// bounds the passes): the final pass is the one the done word names, else the last enqueued
// (k_last); its total goes to tot_final, and its chunk offsets to the caller's array when that
// pass wrote the other one (pass k writes offsets [k & 1]).
__global__ __launch_bounds__(256) void chain_final_kernel(const uint64_t* tot, const uint32_t* done, const uint64_t* off1,
                                                          uint64_t* chunk_off, uint64_t nchunks, uint32_t k_last,
                                                          uint64_t* tot_final) {
    const uint32_t d = __hip_atomic_load(const_cast<uint32_t*>(done), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t k = d ? (d & ~kDoneBytePass) : k_last;
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i == 0) *tot_final = tot[k & 1u];
    if (chunk_off && (k & 1u) && i <= nchunks) chunk_off[i] = off1[i];
}

// ===========================================================================================
// The rest of a general map's chain in one launch (round 4).  Once a pass leaves chunks small,
// a u16 pass is mostly fixed cost (launch, chunk map, tickets, a look-back round trip; 11-18 us on
// a few thousand tokens), and a 24-level chain paid it 14 times.  finish_chunks_kernel takes a
// group of consecutive chunks per workgroup, holds their tokens in LDS and runs greedy passes over
// them until one merges nothing (tokenizer.rs:63-86 per chunk: a pass that merges nothing in a
// chunk leaves it as it is, so running the group to its fixpoint runs every chunk to its own), then
// places the group's final tokens by a decoupled look-back over the groups' token counts.  Chunk
// ends cut pairs as in the other passes (a chunk's first token always lands).
//
// In place: a group writes its final tokens only after its look-back, i.e. after every earlier
// group published its count, which each does after reading its input into LDS; and it writes below
// the next group's input (final prefixes never exceed the input's).  Groups come from a ticket, so
// the lowest unfinished group always has a running workgroup.
//
// finish_gate_kernel runs first: it checks every group fits in LDS (else the finish kernel returns
// at once and the ordinary passes the host enqueued behind it run), zeroes the groups' status
// words and the ticket.  Both return at once when an earlier pass was final.
// ===========================================================================================
constexpr uint32_t kFinThreads = 1024;
constexpr uint32_t kFinCap = kFinThreads * 16;   // tokens of a group in LDS (one 16-token segment per lane)
constexpr uint32_t kFinMaxChunks = 1024;         // chunks per group

// Chunks per group from the longest chunk (the gate's word): as many as surely fit in LDS together.
__device__ __forceinline__ uint32_t fin_group_of(uint32_t lmax) {
    const uint32_t g = kFinCap / (lmax ? lmax : 1u);
    return g < 1u ? 1u : (g > kFinMaxChunks ? kFinMaxChunks : g);
}

// One thread per chunk: the longest chunk into the gate word (capped at kFinCap + 1: too long),
// the chunk's group status word zeroed (groups never outnumber chunks), the ticket zeroed.
__global__ __launch_bounds__(256) void finish_gate_kernel(PassParams p) {
    if (seg::pass_done(p)) return;
    const uint64_t c = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (c == 0) p.ctl[0] = 0u;
    if (c >= p.nchunks) return;
    p.status[c] = 0ull;
    const uint64_t len = p.cstart[c + 1] - p.cstart[c];
    atomicMax(p.fin_gate, (uint32_t)(len > kFinCap ? kFinCap + 1u : len));
}

// Look-back over the groups before g (one wave): windows of 64 status words, the counts of the
// aggregates in front of the nearest inclusive prefix summed with a butterfly of lane shuffles.
// Every group function is "carry 1, n tokens", so no carry chain is needed.
__device__ __forceinline__ void fin_lookback(const PassParams& p, uint64_t g, int lane, uint32_t& C, uint64_t& O,
                                             uint32_t& how, uint32_t& spins) {
    int64_t k = (int64_t)g - 1;
    uint64_t acc = 0;
    uint32_t rounds = 0;
    SpinClock clk;
    for (;;) {
        const int64_t idx = k - lane;
        const uint64_t s = idx >= 0 ? st_read(p.status + idx) : st_incl(1u, 0ull);
        const uint32_t flag = (uint32_t)(s >> 62);
        const uint64_t inc = __ballot(flag == 2u), rdy = __ballot(flag != 0u);
        const int f = inc ? (int)__builtin_ctzll(inc) : 64;
        const uint64_t need = f >= 63 ? ~0ull : ((2ull << f) - 1ull);
        if ((rdy & need) != need) {
            ++spins;
            if (clk.expired()) {
                if (lane == 0) flag_error(p.ctl, KARG(sticky), 1u);
                C = 2u;
                O = 0ull;
                return;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint32_t cnt = lane < f ? (uint32_t)(s & 0x3FFFFFFFull) : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, d, 64);
        acc += cnt;
        if (f < 64) {
            const uint64_t sf = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(s >> 32), f) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)s, f);
            O = acc + (sf & (kStLiveIncl - 1ull));
            C = 1u;
            how = (uint32_t)f | (rounds << 8);
            return;
        }
        k -= 64;
        ++rounds;
    }
}

// Error bit of the finish kernel's invariants (ctl[1]; first-error record: T = group + 1, j = which
// check, O = the group's offset or 0, value = the count that broke it).  Each is checked before the
// write it guards, so a broken count is a flagged BLT_E_IO, never a store outside the group's range:
//   0xF1 the group's input (from the previous pass's chunk offsets) is longer than LDS holds, or its
//        chunk offsets are not increasing
//   0xF2 a pass's count is above its input's, or below half of it (a pass at most halves a chunk)
//   0xF3 the final chunk offsets are not increasing, or end past the group's count
constexpr uint32_t kFinBadBit = 64u;
template <int kHash>
__global__ __launch_bounds__(kFinThreads) void finish_chunks_kernel(PassParams p) {
    extern __shared__ __attribute__((aligned(16))) uint2 s_fhash[];
    __shared__ __attribute__((aligned(16))) uint16_t s_tok[2][kFinCap + 16];
    __shared__ uint32_t s_cpos[2][kFinMaxChunks + 1];   // chunk starts in the group's tokens, [nc] = count
    __shared__ uint32_t s_wfn[kFinThreads / 64][4];
    __shared__ uint32_t s_gin[kFinThreads / 64][2];    // per wave: carry-in, tokens before it
    __shared__ uint32_t s_cnt;
    __shared__ uint32_t s_g;
    __shared__ uint64_t s_O;
    if (seg::pass_done(p)) return;
    const uint32_t lmax = __hip_atomic_load(p.fin_gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lmax > kFinCap) return;   // a chunk too long for LDS: the ordinary passes run
    const uint32_t grp = fin_group_of(lmax);
    const uint64_t ngroups = (p.nchunks + grp - 1) / grp;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kW = kFinThreads / 64;
    if constexpr (kHash != 0) {   // four loads in flight per thread per round (not one)
        const uint4* src = reinterpret_cast<const uint4*>(p.hbuckets);
        uint4* dst = reinterpret_cast<uint4*>(s_fhash);
        const uint32_t nu = p.hbytes / 16u;
        for (uint32_t i0 = 0; i0 < nu; i0 += 4u * kFinThreads) {
            // (indices clamped to the last unit, loads and stores unconditional: a branch per load
            // let the compiler sink each load to its store and wait for it there; the lanes past the
            // end copy the last unit again, the same bytes)
            const uint32_t b = i0 + (uint32_t)tid, last = nu - 1u;
            const uint32_t j0 = b < nu ? b : last, j1 = b + kFinThreads < nu ? b + kFinThreads : last;
            const uint32_t j2 = b + 2u * kFinThreads < nu ? b + 2u * kFinThreads : last;
            const uint32_t j3 = b + 3u * kFinThreads < nu ? b + 3u * kFinThreads : last;
            const uint4 v0 = src[j0], v1 = src[j1], v2 = src[j2], v3 = src[j3];
            dst[j0] = v0; dst[j1] = v1; dst[j2] = v2; dst[j3] = v3;
        }
    }
    const bool inject = (KARG(inject) & kInjectFinish) != 0u;   // test hook: a broken pass count
    // persistent: groups from the ticket, in order, until none is left
    for (;;) {
    __syncthreads();
    if (tid == 0) s_g = atomicAdd(p.ctl, 1u);
    __syncthreads();
    const uint64_t g = s_g;
    if (g >= ngroups) return;
    const uint64_t c0 = g * grp, c1 = c0 + grp < p.nchunks ? c0 + grp : p.nchunks;
    const uint32_t nc = (uint32_t)(c1 - c0);
    const uint64_t S = p.cstart[c0];
    const uint64_t nin64 = p.cstart[c1] - S;
    // the group's input: its chunk offsets increasing, its tokens within LDS (the gate says so; a
    // count that says otherwise is not trusted with the loads and stores below)
    bool ok_in = nin64 <= kFinCap;
    for (uint32_t i = tid; i <= nc; i += kFinThreads) {
        const uint64_t a = p.cstart[c0 + i] - S;
        const uint64_t b = i < nc ? p.cstart[c0 + i + 1] - S : nin64;
        ok_in = ok_in && a <= b && b <= nin64;
        s_cpos[0][i] = (uint32_t)a;
    }
    const uint32_t nin = ok_in ? (uint32_t)nin64 : 0u;
    const uint16_t* in = reinterpret_cast<const uint16_t*>(p.in);
    {   // every load in flight before the first LDS store (a rolled loop waited for each: one
        // global round trip per iteration, 17 of them)
        constexpr uint32_t kPer = (kFinCap + 16 + kFinThreads - 1) / kFinThreads;
        uint16_t t[kPer];
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q) {
            const uint32_t i = (uint32_t)tid + q * kFinThreads;
            t[q] = i < nin ? in[S + i] : (uint16_t)0;
        }
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q) {
            const uint32_t i = (uint32_t)tid + q * kFinThreads;
            if (i < kFinCap + 16) s_tok[0][i] = t[q];
        }
    }
    const uint32_t tab = kHash != 0 ? seg::lds_addr(s_fhash) : 0u;
    uint32_t bad = __syncthreads_or(!ok_in) ? 0xF1u : 0u;   // (uniform)
    uint32_t n = nin;

    uint32_t cur = 0;
    const uint32_t pos0 = 16u * (uint32_t)tid;
    // a wave past the group's tokens looks nothing up (uniform: its first position >= n; a chain's
    // passes halve n, so most waves idle in the later passes).  The skip changes nothing else: such a
    // wave's lanes have no valid position, so every mask below is 0 for them either way.
    for (bool first = true; !bad; first = false) {
        // one greedy pass over s_tok[cur][0, n) into s_tok[cur ^ 1]
        uint32_t x[8];
        {
            const uint4 a = *reinterpret_cast<const uint4*>(&s_tok[cur][pos0]);
            const uint4 b = *reinterpret_cast<const uint4*>(&s_tok[cur][pos0 + 8]);
            x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
        }
        const uint32_t nxt = s_tok[cur][pos0 + 16];
        // pairs (i, i + 1) that may merge: i + 1 < n and i + 1 not a chunk start
        const int32_t rr = (int32_t)n - (int32_t)pos0;
        const uint32_t vmask = rr >= 16 ? 0xFFFFu : (rr <= 0 ? 0u : ((1u << rr) - 1u));
        uint32_t pairs = (vmask >> 1) | (rr > 16 ? 0x8000u : 0u);
        const bool wave_on = 1024u * (uint32_t)wave < n;
        uint32_t a_lo = 0;   // first chunk start >= pos0 + 1 (index into s_cpos)
        if (nc > 1 && wave_on) {
            uint32_t lo = 0, hi = nc;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_cpos[cur][mid] < pos0 + 1u) lo = mid + 1; else hi = mid;
            }
            a_lo = lo;
            for (uint32_t a = lo; a < nc; ++a) {
                const uint32_t b = s_cpos[cur][a];
                if (b > pos0 + 16u) break;
                pairs &= ~(1u << (b - 1u - pos0));
            }
        }
        uint32_t v[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, m = 0;
        if (wave_on) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int h = k >> 1;
                const uint32_t key = (k & 1) ? __builtin_amdgcn_alignbyte(h < 7 ? x[h + 1] : nxt, x[h], 2) : x[h];
                const uint32_t r = seg::tok_get<kHash>(p, tab, key);
                const bool hit = (r >> 31) != 0u && ((pairs >> k) & 1u);
                m |= (uint32_t)hit << k;
                const uint32_t t = hit ? (r & 0xFFFFu) : ((x[h] >> (16 * (k & 1))) & 0xFFFFu);
                if (k & 1) v[h] |= t << 16; else v[h] = t;
            }
        }
        const uint32_t ident = m == 0xFFFFu;
        const uint32_t M1 = merges_for(m, 1u), M0 = merges_for(m, 0u);
        const uint32_t cnt1 = __popc(lands_for(M1, 1u, vmask));
        const uint32_t cnt0 = __popc(lands_for(M0, 0u, vmask));
        const uint32_t cout = ((M1 >> 15) & 1u) ^ 1u;
        uint32_t hasb, bco, excl;
        WaveFn fn;
        resolve_wave(ident, cout, cnt0, cnt1, lane, hasb, bco, excl, fn);
        if (lane == 0) { s_wfn[wave][0] = fn.ident; s_wfn[wave][1] = fn.cout; s_wfn[wave][2] = fn.cnt0; s_wfn[wave][3] = fn.cnt1; }
        __syncthreads();
        if (wave == 0) {
            uint32_t gi = 1, gco = 0, g0 = 0, g1 = 0;
            if (lane < kW) { gi = s_wfn[lane][0]; gco = s_wfn[lane][1]; g0 = s_wfn[lane][2]; g1 = s_wfn[lane][3]; }
            uint32_t ghb, gbc, gex;
            WaveFn tf;
            resolve_wave(gi, gco, g0, g1, lane, ghb, gbc, gex, tf);
            // the group's first token lands (carry-in 1): the high halves
            if (lane < kW) { s_gin[lane][0] = ghb ? gbc : 1u; s_gin[lane][1] = gex >> 16; }
            if (lane == 0) s_cnt = tf.cnt1 + (inject && first ? kFinCap : 0u);
        }
        __syncthreads();
        const uint32_t ncnt = s_cnt;
        // (uniform) a pass keeps at most its input's tokens and at least half of them: any other
        // count would place the stage writes and the group's output by wrong offsets
        if (ncnt > n || 2u * ncnt < n) {
            bad = 0xF2u;   // (s_cnt keeps the count for the record)
            break;
        }
        const uint32_t cg = s_gin[wave][0];
        const uint32_t c = hasb ? bco : cg;
        const uint32_t lane_off = s_gin[wave][1] + (cg ? (excl >> 16) : (excl & 0xFFFFu));
        const uint32_t M = merges_for(m, c);
        const uint32_t L = lands_for(M, c, vmask);
        if (ncnt != n) {   // uniform: something merged
            if (vmask) seg::stage_b16(v, L, seg::lds_addr(&s_tok[cur ^ 1][0]) + 2u * lane_off);
            // chunk starts in [pos0, pos0 + 16) land: their new positions (none past n)
            if (nc > 1 && wave_on) {
                for (uint32_t a = a_lo > 0 ? a_lo - 1 : 0; a < nc; ++a) {
                    const uint32_t b = s_cpos[cur][a];
                    if (b >= pos0 + 16u) break;
                    if (b >= pos0) s_cpos[cur ^ 1][a] = lane_off + __popc(L & ((1u << (b - pos0)) - 1u));
                }
            }
            if (tid == 0) { s_cpos[cur ^ 1][0] = 0u; s_cpos[cur ^ 1][nc] = ncnt; }
        }
        __syncthreads();
        if (ncnt == n) break;   // this pass merged nothing: every chunk of the group is at its fixpoint
        // tokens past the new count must not look like a pair for the next pass's last lanes (masked)
        cur ^= 1;
        n = ncnt;
    }
    if (!bad) {   // the final chunk offsets: increasing, the last one the count
        bool ok = true;
        for (uint32_t i = tid; i < nc; i += kFinThreads) ok = ok && s_cpos[cur][i] <= s_cpos[cur][i + 1];
        if (__syncthreads_or(!ok || s_cpos[cur][nc] != n)) bad = 0xF3u;
    }

    // place the group: its count as an aggregate (constant carry 1: chunks never merge across), the
    // look-back over the groups before it, then its tokens, chunk offsets and (last group) the total.
    // A group that broke an invariant flags it and writes nothing; it publishes its input count so
    // the groups after it still finish (their offsets stay below their own inputs).
    if (wave == 0) {
        uint32_t C = 1u, how = 0, spins = 0;
        uint64_t O = 0;
        const uint32_t cnt = bad ? (uint32_t)(nin64 < (1ull << 30) ? nin64 : (1ull << 30) - 1u) : n;
        if (g == 0) {
            if (lane == 0) st_publish(p.status, st_incl(1u, cnt));
        } else {
            if (lane == 0) st_publish(p.status + g, st_agg(1u, 1u, cnt, cnt));
            if (!bad) {
                fin_lookback(p, g, lane, C, O, how, spins);
                if (lane == 0) {
                    if (C > 1u || O > S) {   // a failed look-back (flagged) or a broken prefix: write nothing
                        if (C <= 1u) record_error(p, 4u, (uint32_t)g, 0xFEu, O, n, C);
                        O = ~0ull;
                    } else {
                        st_publish(p.status + g, st_incl(1u, O + n));
                    }
                }
            }
        }
        if (bad) {
            if (lane == 0) record_error(p, kFinBadBit, (uint32_t)g, bad, S, bad == 0xF2u ? s_cnt : n, nc);
            O = ~0ull;
        }
        if (lane == 0) {
            s_O = O;
            if (p.debug) {   // tests only: the group's record
                uint64_t* d = p.debug + 16ull * g;
                d[0] = g; d[1] = S; d[2] = nin64; d[3] = n; d[4] = O;
                d[5] = C | ((uint64_t)how << 8) | ((uint64_t)spins << 32);
                d[6] = lmax | ((uint64_t)grp << 32); d[7] = nc | ((uint64_t)bad << 32);
                d[8] = g ? st_read(p.status + g - 1) : 0; d[9] = st_read(p.status);
                d[10] = st_read(p.status + g);
                d[11] = g >= 2 ? st_read(p.status + g - 2) : 0;
            }
        }
    }
    __syncthreads();
    const uint64_t O = s_O;
    if (O == ~0ull) continue;
    uint16_t* out = reinterpret_cast<uint16_t*>(p.out);
    for (uint32_t i = tid; i < n; i += kFinThreads) out[O + i] = s_tok[cur][i];
    for (uint32_t i = tid; i < nc; i += kFinThreads) p.chunk_off[c0 + i] = O + s_cpos[cur][i];
    if (c1 == p.nchunks && tid == 0) {
        p.chunk_off[p.nchunks] = O + n;
        *p.total = O + n;
        *p.done = p.pass_id;
    }
    }   // groups
}

__global__ void inject_error_kernel(uint32_t* ctl, uint32_t* sticky) {
    if (threadIdx.x == 0) flag_error(ctl, sticky, 1u);
}

// ---- launchers ---------------------------------------------------------------------------
// Persistent-grid size of a kernel on a device: CUs x resident workgroups per CU, queried once
// per (device, kernel) and cached in atomics (launchers run concurrently from many host threads).
struct GridCache {
    std::atomic<int> cus[64];
    std::atomic<int> occ[64][16];
};
static GridCache g_grid;   // zero-initialised (static storage)
static int grid_for(uint32_t ntiles, int device, const void* fn, int threads, int kernel_id) {
    int cus = 0, occ = 0;
    if (device >= 0 && device < 64) {
        cus = g_grid.cus[device].load(std::memory_order_relaxed);
        occ = g_grid.occ[device][kernel_id].load(std::memory_order_relaxed);
    }
    if (!cus) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) cus = 1;
        if (device >= 0 && device < 64) g_grid.cus[device].store(cus, std::memory_order_relaxed);
    }
    if (!occ) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, threads, 0) != hipSuccess || occ < 1) occ = 1;
        if (device >= 0 && device < 64) g_grid.occ[device][kernel_id].store(occ, std::memory_order_relaxed);
    }
    long long g = (long long)cus * occ;
    if (g > (long long)ntiles) g = ntiles;
    return (int)(g < 1 ? 1 : g);
}

// The same for a kernel whose occupancy depends on its dynamic LDS (the u16 pass with the map's
// bucket table in LDS): cached per (device, kernel, bytes), so a chain of passes queries once.
static std::mutex g_grid_mu;
static std::unordered_map<uint64_t, int> g_grid_smem;
static int grid_for_smem(uint32_t ntiles, int device, const void* fn, int threads, size_t smem) {
    const uint64_t key = ((uint64_t)(uint32_t)device << 40) ^ ((uint64_t)(uintptr_t)fn << 20) ^ (uint64_t)smem;
    int g = 0;
    {
        std::lock_guard<std::mutex> lk(g_grid_mu);
        auto it = g_grid_smem.find(key);
        if (it != g_grid_smem.end()) g = it->second;
    }
    if (!g) {
        int cus = 0, occ = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) cus = 1;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, threads, smem) != hipSuccess || occ < 1) occ = 1;
        g = cus * occ;
        std::lock_guard<std::mutex> lk(g_grid_mu);
        g_grid_smem[key] = g;
    }
    if ((uint64_t)g > ntiles) g = (int)ntiles;
    return g < 1 ? 1 : g;
}

hipError_t launch_merge_pass(const PassParams& p, int input_u16, int big_endian, int device, hipStream_t s) {
    if (p.ntiles == 0) return hipSuccess;
    if (!input_u16) {
        const void* fn = big_endian ? (const void*)merge_pass_kernel<uint8_t, true> : (const void*)merge_pass_kernel<uint8_t, false>;
        const int grid = grid_for(p.ntiles, device, fn, kThreads, big_endian ? 1 : 0);
        if (big_endian) hipLaunchKernelGGL((merge_pass_kernel<uint8_t, true>), dim3(grid), dim3(kThreads), 0, s, p);
        else hipLaunchKernelGGL((merge_pass_kernel<uint8_t, false>), dim3(grid), dim3(kThreads), 0, s, p);
        return hipGetLastError();
    }
    // u16 passes: big-endian in and out; the bucket table in LDS when it fits (then several
    // workgroups share a CU and cover each other's barriers).  p.ntiles is the upper bound the
    // input size allows; the kernel reads the actual count from p.n_dev.
    const bool lds = p.hbytes <= kHashLdsMax;
    const void* fn = lds ? (const void*)merge_tokens_kernel<true> : (const void*)merge_tokens_kernel<false>;
    const size_t smem = lds ? p.hbytes : 0;
    const int grid = grid_for_smem(p.ntiles, device, fn, kThreads, smem);
    if (lds) hipLaunchKernelGGL((merge_tokens_kernel<true>), dim3((unsigned)grid), dim3(kThreads), smem, s, p);
    else hipLaunchKernelGGL((merge_tokens_kernel<false>), dim3((unsigned)grid), dim3(kThreads), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_scan_bytes(const PassParams& p, int mode, int live, int device, hipStream_t s) {
    if (p.ntiles == 0) return hipSuccess;
    using seg::scan_bytes_kernel;
    const void* fn = mode == 0 ? (const void*)scan_bytes_kernel<true, 0, false>
                     : mode == 1 ? (live ? (const void*)scan_bytes_kernel<true, 1, true> : (const void*)scan_bytes_kernel<true, 1, false>)
                                 : (live ? (const void*)scan_bytes_kernel<true, 2, true> : (const void*)scan_bytes_kernel<true, 2, false>);
    if (mode < 0 || mode > 2 || (mode == 0 && live)) return hipErrorInvalidValue;
    // every byte-pass instantiation holds the whole LDS: one workgroup per CU, one cache entry
    const int grid = grid_for(p.ntiles, device, fn, seg::kThreads, 4);
    const dim3 g((unsigned)grid), b(seg::kThreads);
    if (mode == 0) hipLaunchKernelGGL((scan_bytes_kernel<true, 0, false>), g, b, 0, s, p);
    else if (mode == 1 && live) hipLaunchKernelGGL((scan_bytes_kernel<true, 1, true>), g, b, 0, s, p);
    else if (mode == 1) hipLaunchKernelGGL((scan_bytes_kernel<true, 1, false>), g, b, 0, s, p);
    else if (live) hipLaunchKernelGGL((scan_bytes_kernel<true, 2, true>), g, b, 0, s, p);
    else hipLaunchKernelGGL((scan_bytes_kernel<true, 2, false>), g, b, 0, s, p);
    return hipGetLastError();
}

hipError_t launch_scan_tokens(const PassParams& p, int map_ready, int device, hipStream_t s) {
    if (p.n == 0) return hipSuccess;
    // p.n bounds the token count the kernels read from p.n_dev
    const uint64_t ranges = (p.n + kTokRange - 1) / kTokRange;
    if (!map_ready) hipLaunchKernelGGL(seg::chunk_map_kernel, dim3((unsigned)((ranges + 255) / 256)), dim3(256), 0, s, p);
    const bool lds = p.hbytes <= kHashLdsMax;
    const int mode = lds ? (p.hone ? 2 : 1) : 0;
    const void* fn = mode == 2 ? (const void*)seg::scan_tokens_kernel<2>
                     : mode == 1 ? (const void*)seg::scan_tokens_kernel<1> : (const void*)seg::scan_tokens_kernel<0>;
    const uint32_t ntiles = (uint32_t)((p.n + kTilePosTok - 1) / kTilePosTok);
    const int grid = grid_for(ntiles, device, fn, seg::kThreads, 5 + mode);
    const size_t smem = lds ? ((size_t)p.hbytes + 1023) & ~(size_t)1023 : 0;   // whole KiB (LDS-DMA rows)
    const dim3 g((unsigned)grid), b(seg::kThreads);
    if (mode == 2) hipLaunchKernelGGL((seg::scan_tokens_kernel<2>), g, b, smem, s, p);
    else if (mode == 1) hipLaunchKernelGGL((seg::scan_tokens_kernel<1>), g, b, smem, s, p);
    else hipLaunchKernelGGL((seg::scan_tokens_kernel<0>), g, b, 0, s, p);
    return hipGetLastError();
}

hipError_t launch_scan_fused(const PassParams& p, int device, hipStream_t s) {
    if (p.n == 0) return hipSuccess;
    if (p.hbytes > kHashLdsMax || p.cs < kMinChunkBytes || !p.fused_fail) return hipErrorInvalidValue;
    const int mode = p.hone ? 2 : 1;
    const void* fn = mode == 2 ? (const void*)seg::scan_tokens_kernel<2, true> : (const void*)seg::scan_tokens_kernel<1, true>;
    const uint32_t ntiles = (uint32_t)((p.n + kTilePosTok - 1) / kTilePosTok);
    const int grid = grid_for(ntiles, device, fn, seg::kThreads, 8 + mode);
    const size_t smem = ((size_t)p.hbytes + 1023) & ~(size_t)1023;
    const dim3 g((unsigned)grid), b(seg::kThreads);
    if (mode == 2) hipLaunchKernelGGL((seg::scan_tokens_kernel<2, true>), g, b, smem, s, p);
    else hipLaunchKernelGGL((seg::scan_tokens_kernel<1, true>), g, b, smem, s, p);
    return hipGetLastError();
}

hipError_t launch_basic_expand(const uint8_t* in, uint64_t n, uint8_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n / 8 + 255) / 256;    // one 8-byte block per thread
    if (blocks < 1) blocks = 1;
    if (blocks > kBasicMaxBlocks) blocks = kBasicMaxBlocks;
    hipLaunchKernelGGL(basic_expand_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, n, out);
    return hipGetLastError();
}

hipError_t launch_chain_final(const uint64_t* tot, const uint32_t* done, const uint64_t* off1, uint64_t* chunk_off,
                              uint64_t nchunks, uint32_t k_last, uint64_t* tot_final, hipStream_t s) {
    const uint64_t blocks = chunk_off ? (nchunks + 1 + 255) / 256 : 1;
    hipLaunchKernelGGL(chain_final_kernel, dim3((unsigned)blocks), dim3(256), 0, s, tot, done, off1, chunk_off, nchunks,
                       k_last, tot_final);
    return hipGetLastError();
}

hipError_t launch_finish(const PassParams& p, int device, hipStream_t s) {
    if (p.nchunks == 0 || !p.fin_gate || p.nchunks > 0xFFFFFFFFull * 256u) return hipErrorInvalidValue;
    hipLaunchKernelGGL(finish_gate_kernel, dim3((unsigned)((p.nchunks + 255) / 256)), dim3(256), 0, s, p);
    const bool lds = p.hbytes <= kHashLdsMax;
    const int mode = lds ? (p.hone ? 2 : 1) : 0;
    const size_t smem = lds ? (size_t)p.hbytes : 0;
    // persistent: one workgroup per CU (its LDS), no more than there are chunks
    const void* fn = mode == 2 ? (const void*)finish_chunks_kernel<2>
                     : mode == 1 ? (const void*)finish_chunks_kernel<1> : (const void*)finish_chunks_kernel<0>;
    const int grid = grid_for_smem((uint32_t)std::min<uint64_t>(p.nchunks, 0xFFFFFFFFull), device, fn, kFinThreads, smem);
    const dim3 g((unsigned)grid), b(kFinThreads);
    if (mode == 2) hipLaunchKernelGGL((finish_chunks_kernel<2>), g, b, smem, s, p);
    else if (mode == 1) hipLaunchKernelGGL((finish_chunks_kernel<1>), g, b, smem, s, p);
    else hipLaunchKernelGGL((finish_chunks_kernel<0>), g, b, 0, s, p);
    return hipGetLastError();
}

// ===========================================================================================
// Sparse passes of a cyclic general map (round 4).  After a chain's first u16 passes a cyclic map's
// passes merge almost nothing (self-valued merges on text: 59,215, 460, 16, 2 merges per 2 MiB over
// four passes), yet each full pass rewrites every token behind its first merge.  Here the tokens stay
// in place: a merge writes its value at its first position and marks the consumed one in a hole
// bitmap, and a pass touches only the maximal runs of mergeable pairs.  Why that is the greedy pass
// (tokenizer.rs:63-86): a run's first position lands (the pair before it does not merge, or it starts
// a chunk), and inside a run every pair merges, so the pass merges its pairs from the first position
// on, alternately; everywhere else every position lands and emits itself.  Which runs: in pass k + 1
// a mergeable pair has a token pass k made (two tokens both left alone by pass k were next to each
// other in its input too, and the first landed without merging: the pair was looked up and rejected,
// or cut at a chunk end), and only a live one (a key component) can be in a key.  So pass k's live
// new tokens are the seeds of pass k + 1, and the first sparse pass takes every mergeable pair as a
// seed (sparse_detect_kernel).  A run is processed by the thread of its leftmost seed: walking left,
// a thread that meets another seed in the run leaves it.  Passes read only (the merges and next seeds
// go to lists); a second kernel applies the merges, so no thread sees another's writes.  A run ends
// at the first pair that does not merge, also right after a merge: the greedy walk then lands on the
// next position anyway, but that position's pair belongs to the next run and its owner.
// (tools/sparse_sim.py restates these passes sequentially against the oracle.)
// ===========================================================================================
__device__ __forceinline__ uint32_t sp_lookup(const SparseParams& q, uint32_t key) {
    const uint2 x = q.hbuckets[bucket_hash(key, q.hmul1, q.hshift)];
    const uint2 y = q.hbuckets[bucket_hash(key, q.hmul2, q.hshift)];
    return (x.x == key ? x.y : 0u) | (y.x == key ? y.y : 0u);
}
__device__ __forceinline__ bool sp_bit(const uint32_t* b, uint64_t p) { return ((b[p >> 5] >> (p & 31u)) & 1u) != 0u; }
__device__ __forceinline__ int64_t sp_prev(const SparseParams& q, int64_t p) {   // previous non-hole, or -1
    for (--p; p >= 0 && sp_bit(q.holes, (uint64_t)p); --p) {}
    return p;
}
__device__ __forceinline__ uint64_t sp_next(const SparseParams& q, uint64_t p) {   // next non-hole, or n
    for (++p; p < q.n && sp_bit(q.holes, p); ++p) {}
    return p;
}
__device__ __forceinline__ uint32_t sp_key(const SparseParams& q, uint64_t a, uint64_t b) {
    return (uint32_t)q.tok[a] | ((uint32_t)q.tok[b] << 16);
}

// Every sparse kernel is enqueued without a host read: it returns when the gate word is set (the
// chain ended, or the fused kernel must fall back) and reads the token count from the device.  The
// compaction kernels also return when the detect kernel's seeds overflowed (nothing was applied) or
// when their condition word is nonzero (the passes before them have not converged: the host runs
// more passes first).
__device__ __forceinline__ bool sp_gated(const SparseParams& q) { return q.gate && *q.gate != 0ull; }
__device__ __forceinline__ bool sp_compact_skip(const SparseParams& q, const uint32_t* nseeds0) {
    (void)nseeds0;
    return sp_gated(q) || (*q.flags & 2u) != 0u || (q.cond && *q.cond != 0u);
}

// Every position whose pair with the next one is a merge (not across a chunk start): the first
// sparse pass's seeds, as a bitmap (bits_in; the first pass reads its seeds from it, so no list and
// no atomics here: one append per wave that had seeds serialised on the counter's address, 561 us
// on selfval's ~60 K seeds).  A lane takes 32 aligned positions (64 bytes of tokens, one word of each bitmap,
// stored whole: the seed bitmap, the holes and the later passes' two seed bitmaps zeroed); the next
// lane's first token comes by DPP.  The bucket table is staged in LDS when it fits (kLds).
// The detect gate: block b counts the mergeable pairs among 8192 positions from b n / 64 (chunk
// starts ignored: an estimate), one atomic per block.
__global__ __launch_bounds__(1024) void sparse_sample_kernel(SparseParams q) {
    __shared__ uint32_t s_w[16];
    if (sp_gated(q)) return;
    // the run's counters and per-tile words zeroed (every later sparse kernel runs behind this one)
    for (uint32_t i = blockIdx.x * 1024u + threadIdx.x; i < q.zero16; i += kSparseSampleBlocks * 1024u)
        q.zero[i] = make_uint4(0u, 0u, 0u, 0u);
    const uint64_t n = *q.n_dev;
    // 8 positions per thread: one 16-byte load and 8 independent lookups (a loop of dependent
    // lookups per thread took 9.5 us)
    const uint64_t p0 = n <= kSparseSample ? (uint64_t)blockIdx.x * 8192u
                                           : ((n - 8192u) / (kSparseSampleBlocks - 1u) * blockIdx.x) & ~7ull;
    const uint64_t i0 = p0 + 8ull * threadIdx.x;
    uint32_t t[9];
    if (i0 + 9 <= n) {
        const uint4 v = *reinterpret_cast<const uint4*>(q.tok + i0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) t[k] = (w[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
        t[8] = q.tok[i0 + 8];
    } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) t[k] = i0 + k < n ? q.tok[i0 + k] : 0u;
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (i0 + k + 1 < n) cnt += sp_lookup(q, t[k] | (t[k + 1] << 16)) >> 31;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, d, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) tot += s_w[k];
        q.sample[blockIdx.x] = tot;
    }
}

// Bitmap words per workgroup of sparse_list_kernel (whole rounds of 4096, at most kListBlocks
// workgroups).
constexpr uint32_t kListWords = 16 * 256, kListBlocks = 512;
__host__ __device__ __forceinline__ uint64_t sp_list_words(uint64_t nwords) {   // bitmap words per workgroup
    const uint64_t r = (nwords + (uint64_t)kListBlocks * kListWords - 1) / ((uint64_t)kListBlocks * kListWords);
    return (r ? r : 1ull) * kListWords;
}

constexpr uint64_t kDetectCsLds = 2048;   // chunk starts the detect kernel stages in LDS (16 KiB)
template <bool kLds>
__global__ __launch_bounds__(256) void sparse_detect_kernel(SparseParams qa) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    if (sp_gated(qa)) return;
    SparseParams q = qa;
    q.n = *qa.n_dev;
    {   // the gate: more seeds predicted than half the lists hold, not taken
        const uint64_t sampled = q.n < kSparseSample ? q.n : kSparseSample;
        uint32_t smp = q.sample[threadIdx.x & 63];   // (kSparseSampleBlocks = 64 words)
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) smp += (uint32_t)__shfl_xor((int)smp, d, 64);
        if ((uint64_t)smp * q.n > (uint64_t)(q.cap / 2) * sampled) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(q.flags, 3u);
            return;
        }
    }
    const int lane = threadIdx.x & 63;
    const uint2* tab = q.hbuckets;
    // the chunk starts in LDS after the table (up to kDetectCsLds of them): each wave's binary
    // search then costs LDS round trips, not global ones (four dependent loads per wave on selfval's
    // 16 chunks, longer than the wave's own token loads)
    const bool cs_lds = q.nchunks <= kDetectCsLds;
    uint64_t* const s_cs = reinterpret_cast<uint64_t*>(s_dyn + (kLds ? ((q.hbytes + 15u) & ~15u) / 4u : 0u));
    if (kLds || cs_lds) {
        if (kLds) {
            const uint32_t nw = q.hbytes / 4;
            const uint32_t* src = reinterpret_cast<const uint32_t*>(q.hbuckets);
            for (uint32_t w = threadIdx.x; w < nw; w += 256) s_dyn[w] = src[w];
        }
        if (cs_lds)
            for (uint32_t i = threadIdx.x; i < q.nchunks; i += 256) s_cs[i] = q.coff_in[i];
        __syncthreads();
    }
    const uint64_t* const cs = cs_lds ? s_cs : q.coff_in;
    auto lookup = [&](uint32_t key) -> uint32_t {
        const uint32_t b1 = bucket_hash(key, q.hmul1, q.hshift);
        const uint2 x = kLds ? reinterpret_cast<const uint2*>(s_dyn)[b1] : tab[b1];
        uint32_t v = x.x == key ? x.y : 0u;
        if (!q.hone) {
            const uint32_t b2 = bucket_hash(key, q.hmul2, q.hshift);
            const uint2 y = kLds ? reinterpret_cast<const uint2*>(s_dyn)[b2] : tab[b2];
            v |= y.x == key ? y.y : 0u;
        }
        return v;
    };
    const uint64_t nwords = (q.n + 31) / 32;
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t base = (uint64_t)blockIdx.x * 256u + (uint64_t)(threadIdx.x & ~63u); base < nwords; base += stride) {
        const uint64_t wd = base + (uint64_t)lane;   // the loop is wave-uniform; lanes past the end add nothing
        const uint64_t i0 = wd * 32;
        uint32_t w[16];
        if (i0 + 32 <= q.n) {
            const uint4* src = reinterpret_cast<const uint4*>(q.tok + i0);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 v = src[k];
                w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t lo = i0 + 2u * k < q.n ? q.tok[i0 + 2u * k] : 0u;
                const uint32_t hi = i0 + 2u * k + 1u < q.n ? q.tok[i0 + 2u * k + 1u] : 0u;
                w[k] = lo | (hi << 16);
            }
        }
        // the chunk starts in the wave's 2048 positions and the one after (wave-uniform: a binary
        // search over the sorted chunk starts, then the few in range): this lane's chunk-start
        // bits, and whether position i0 + 32 starts a chunk
        const uint64_t W0 = base * 32;
        uint64_t lo = 0, hi = q.nchunks;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (cs[mid] < W0) lo = mid + 1;
            else hi = mid;
        }
        uint32_t csw = 0, nc = 0;
        for (uint64_t c = lo; c < q.nchunks; ++c) {
            const uint64_t p = cs[c];
            if (p > W0 + 2048) break;
            if (p >= i0 && p < i0 + 32) csw |= 1u << (uint32_t)(p - i0);
            nc |= p == i0 + 32 ? 1u : 0u;
        }
        // lane + 1's first token (wave_shl:1); lane 63 reads it
        uint32_t nt = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(w[0] & 0xFFFFu), 0x130, 0xF, 0xF, false);
        if (lane == 63) nt = i0 + 32 < q.n ? q.tok[i0 + 32] : 0u;
        if (wd < nwords) {
            uint32_t mask = 0;
            const uint32_t cut = (csw >> 1) | (nc << 31);   // bit k: position k + 1 starts a chunk
#pragma unroll
            for (int k = 0; k < 32; ++k) {
                const uint32_t a = (w[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                const uint32_t b = k < 31 ? (w[(k + 1) >> 1] >> (16 * ((k + 1) & 1))) & 0xFFFFu : nt;
                if (i0 + k + 1 < q.n && ((cut >> k) & 1u) == 0u && (lookup(a | (b << 16)) >> 31)) mask |= 1u << k;
            }
            q.bits_in[wd] = mask;   // the bitmaps of these positions, written whole (no memsets)
            q.bits_out[wd] = 0u;
            q.bits_alt[wd] = 0u;
            q.holes[wd] = 0u;
        }
    }
}

// The first pass's seed list from the detect kernel's bitmap.  A workgroup per kListBlocks-th of
// the bitmap (whole rounds of 4096 words; 16 consecutive words per thread and round, four 16-byte
// loads): it counts its seeds, publishes the count in its status word, and sums the published
// counts of the workgroups before it (at most kListBlocks - 1 words, read at once by its threads):
// its place in the list.  Its seeds then go out in position order, one workgroup scan per round.
// Its block comes from a ticket, so every count waited for is published by a running or finished
// workgroup.  (A first pass that reads its bitmap directly, a lane per word,
// measured 549 us on selfval against 20 us from this list: a lane walks its word's seeds one after
// another, and a long run's seeds sit in few words.  On selfval: rounds of 256 words and one atomic
// per workgroup on the list's counter, 45 us; one round, 31 us (the atomics serialise, ~11 ns each
// on one word: tools/atomic_probe.hip); a look-back over 64 predecessors per round trip, 18.5 us
// (every workgroup is resident at once, so inclusive prefixes spread slowly); counts added by the
// detect kernel, 11 us here but +20-24 us there.)  The status words are the compaction's (zeroed
// with the run's counters); the move kernel later marks them with another bit.
constexpr uint64_t kListPub = 1ull << 62;   // a list workgroup's count is published
__global__ __launch_bounds__(256) void sparse_list_kernel(SparseParams qa) {
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_pre[4];
    __shared__ uint32_t s_bad, s_b;
    if (sp_gated(qa)) return;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // (the detect gate: not taken) read once for the workgroup: another workgroup of this kernel may
    // set the flags meanwhile, and every wave must reach the barriers below.  The workgroup's block
    // of words from a ticket (round 6): the counts it waits for are those of lower tickets, whose
    // workgroups have started and publish theirs before waiting for anything (no reliance on the
    // order workgroups are dispatched in; at most kListBlocks atomics).
    if (tid == 0) {
        s_bad = *qa.flags & 2u;
        s_b = s_bad ? 0u : atomicAdd(qa.super_cnt + 1, 1u);   // (zeroed with the run's counters)
    }
    __syncthreads();
    if (s_bad) return;
    const uint32_t b = s_b;
    // words per workgroup from the host's bound qa.n, as the launcher sized the grid with (from the
    // device's count, which may cross a round boundary the bound does not, the grid could fall short)
    const uint64_t nwords = (*qa.n_dev + 31) / 32, per = sp_list_words((qa.n + 31) / 32);
    const uint64_t wb0 = (uint64_t)b * per, wb1 = wb0 + per < nwords ? wb0 + per : nwords;
    if (wb0 >= nwords) return;   // (uniform; no later workgroup has words either)
    auto load16 = [&](uint64_t w0, uint32_t (&m)[16]) {
        if (w0 + 16 <= wb1) {   // (the bitmaps are 16-byte aligned)
            const uint4* src = reinterpret_cast<const uint4*>(qa.bits_in + w0);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 v = src[k];
                m[4 * k] = v.x; m[4 * k + 1] = v.y; m[4 * k + 2] = v.z; m[4 * k + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) m[k] = w0 + k < wb1 ? qa.bits_in[w0 + k] : 0u;
        }
    };
    auto popc16 = [](const uint32_t (&m)[16]) {
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) c += (uint32_t)__popc(m[k]);
        return c;
    };
    // this workgroup's count (the first round stays in registers)
    uint32_t m[16];
    load16(wb0 + 16ull * tid, m);
    const uint32_t c0 = popc16(m);
    uint32_t call = c0;
    for (uint64_t r0 = wb0 + kListWords; r0 < wb1; r0 += kListWords) {
        uint32_t t[16];
        load16(r0 + 16ull * tid, t);
        call += popc16(t);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) call += (uint32_t)__shfl_xor((int)call, d, 64);
    if (lane == 0) s_w[wave] = call;
    __syncthreads();   // (s_bad is 0 here)
    if (tid == 0) st_publish(qa.status + b, kListPub | (uint64_t)(s_w[0] + s_w[1] + s_w[2] + s_w[3]));
    // the counts before this workgroup
    uint32_t pre = 0;
    bool bad = false;
    for (uint32_t k = tid; k < b; k += 256) {
        uint64_t v = st_read(qa.status + k);
        SpinClock clk;
        while ((v & kListPub) == 0ull) {
            if (clk.expired()) { bad = true; break; }
            __builtin_amdgcn_s_sleep(1);
            v = st_read(qa.status + k);
        }
        pre += (uint32_t)v;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) pre += (uint32_t)__shfl_xor((int)pre, d, 64);
    if (lane == 0) s_pre[wave] = pre;
    if (bad) s_bad = 1u;
    __syncthreads();
    if (s_bad) {   // (never expected) dropped as an overflow: the host's passes take over
        if (tid == 0) atomicOr(qa.flags, 3u);
        return;
    }
    uint32_t base = s_pre[0] + s_pre[1] + s_pre[2] + s_pre[3];
    if (wb1 == nwords && tid == 0) *qa.nseeds_out = base + s_w[0] + s_w[1] + s_w[2] + s_w[3];   // the list's length
    for (uint64_t r0 = wb0; r0 < wb1; r0 += kListWords) {   // (uniform)
        const uint64_t w0 = r0 + 16ull * tid;
        if (r0 != wb0) load16(w0, m);
        const uint32_t c = r0 == wb0 ? c0 : popc16(m);
        const uint32_t incl = wave_incl_scan(c, (int)lane);
        __syncthreads();   // (s_w of the round before read)
        if (lane == 63) s_w[wave] = incl;
        __syncthreads();
        uint32_t o = base + incl - c;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) o += k < wave ? s_w[k] : 0u;
        base += s_w[0] + s_w[1] + s_w[2] + s_w[3];
        if (c) {
            for (int k = 0; k < 16; ++k) {
                for (uint32_t mm = m[k]; mm; mm &= mm - 1u, ++o) {
                    if (o < qa.cap) qa.seeds_out[o] = (uint32_t)(32ull * (w0 + k) + (uint64_t)__builtin_ctz(mm));
                    else atomicOr(qa.flags, 3u);
                }
            }
        }
    }
}

// One sparse pass: the runs of the seeds' owners, merges and next seeds into lists.  The first pass
// takes its seeds from the flat list of sparse_list_kernel (a wave per 64 entries, grid-stride), the
// later ones from the slice the same wave of the pass before filled.  The lanes of a wave walk their
// runs in step, one merge per lane per step, and append each step's merges and new seeds to the
// wave's own slice of each list (wave w: entries [w slice, (w + 1) slice)), counted in registers; the
// wave stores its counts at the end.  (Appending to one list with one atomic per wave step on its
// counter cost ~11 ns per step, serialised on the word: ~20 us for the first pass on selfval.)  A
// slice that overflows sets the flags (bit 2 in the first pass: nothing is applied and the compaction
// does not run, the tokens stay as they were) and the pass's merge total to cap + 1.
__global__ __launch_bounds__(256) void sparse_region_kernel(SparseParams qa) {
    extern __shared__ __attribute__((aligned(16))) uint64_t s_rcs[];   // the chunk starts (kDetectCsLds)
    SparseParams q = qa;
    if (q.nchunks <= kDetectCsLds) {   // (before the flags test: other workgroups may set the flags
                                       // meanwhile, and every wave must reach the barrier)
        for (uint32_t i = threadIdx.x; i < q.nchunks; i += 256) s_rcs[i] = q.coff_in[i];
        __syncthreads();
        q.coff_in = s_rcs;   // (a seed's chunk: binary search in LDS)
    }
    if (sp_gated(qa) || *qa.flags) return;
    q.n = *qa.n_dev;
    const uint32_t oflag = q.first_pass ? 3u : 1u;
    const int lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * 4u + (threadIdx.x >> 6);   // this wave's slice
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t* const mslice = q.merges + 3ull * w * q.slice;
    uint32_t* const sslice = q.seeds_out + (uint64_t)w * q.slice;
    uint32_t nm = 0, nsd = 0;   // merges and next seeds of this wave so far (uniform)
    const bool flat = q.cnt_in == nullptr;
    const uint32_t* const src = flat ? q.seeds_in : q.seeds_in + (uint64_t)w * q.slice;
    const uint32_t ns = flat ? min(*q.nseeds_in, q.cap) : min(q.cnt_in[w], q.slice);
    const uint32_t b0 = flat ? w * 64u : 0u, bstep = flat ? q.nslices * 64u : 64u;
    bool over = false;
    for (uint32_t base = b0; base < ns; base += bstep) {   // (uniform)
        const uint32_t idx = base + (uint32_t)lane;
        // this lane's seed (one list entry), if any
        uint32_t pend = 0;
        uint64_t pbase = 0;
        if (idx < ns) {
            pend = 1u;
            pbase = src[idx];
        }
        bool act = false;
        uint64_t i = 0, c1 = 0;
        while (__ballot(act || pend != 0u) != 0ull) {   // (uniform)
            if (!act && pend != 0u) {   // the seed: its run's first position, if this lane owns it
                const uint64_t sd = pbase + (uint64_t)__builtin_ctz(pend);
                pend &= pend - 1u;
                if (sd < q.n && !sp_bit(q.holes, sd)) {   // (always: a seed is a token)
                    // the seed's chunk [c0, c1): the last chunk start <= sd (binary search)
                    uint64_t lo = 0, hi = q.nchunks;
                    while (hi - lo > 1) {
                        const uint64_t mid = (lo + hi) >> 1;
                        if (q.coff_in[mid] <= sd) lo = mid;
                        else hi = mid;
                    }
                    const uint64_t c0 = q.coff_in[lo];
                    c1 = lo + 1 < q.nchunks ? q.coff_in[lo + 1] : q.n;
                    uint64_t a = sd;
                    bool owner = true;
                    for (;;) {
                        if (a == c0) break;
                        const int64_t pq = sp_prev(q, (int64_t)a);
                        if (pq < 0 || (sp_lookup(q, sp_key(q, (uint64_t)pq, a)) >> 31) == 0u) break;
                        if (sp_bit(q.bits_in, (uint64_t)pq)) { owner = false; break; }   // an earlier seed owns the run
                        a = (uint64_t)pq;
                    }
                    act = owner;
                    i = a;
                }
            }
            // one greedy step from the run's first position, which lands
            uint64_t j = 0;
            uint32_t v = 0;
            if (act) {
                j = sp_next(q, i);
                if (j < c1) v = sp_lookup(q, sp_key(q, i, j));
            }
            const bool mg = act && (v >> 31) != 0u, lv = mg && ((v >> 30) & 1u);
            const uint64_t mm = __ballot(mg), lm = __ballot(lv);
            if (mg) {
                const uint32_t m = nm + (uint32_t)__popcll(mm & below);
                if (m < q.slice) {
                    mslice[3u * m] = (uint32_t)i;
                    mslice[3u * m + 1u] = (uint32_t)j;
                    mslice[3u * m + 2u] = v & 0xFFFFu;
                } else {
                    over = true;
                }
            }
            if (lv) {   // a live token: a seed of the next pass
                const uint32_t so = nsd + (uint32_t)__popcll(lm & below);
                if (so < q.slice) sslice[so] = (uint32_t)i;
                else over = true;
                atomicOr(&q.bits_out[i >> 5], 1u << (i & 31u));
            }
            nm += (uint32_t)__popcll(mm);
            nsd += (uint32_t)__popcll(lm);
            if (act) {
                act = false;
                if (mg) {
                    const uint64_t k = sp_next(q, j);
                    // k lands; the run goes on only if (j, k) merges: else k starts the next run, whose
                    // own leftmost seed takes it (k's pair may merge, and two lanes would both make it)
                    if (k < c1 && (sp_lookup(q, sp_key(q, j, k)) >> 31) != 0u) {
                        i = k;
                        act = true;
                    }
                }
            }
        }
    }
    if (lane == 0) {
        q.cnt_merges[w] = min(nm, q.slice);
        q.cnt_seeds[w] = min(nsd, q.slice);
    }
    if (__ballot(over) != 0ull && lane == 0) {
        atomicOr(q.flags, oflag);
        *q.nmerges = q.cap + 1u;   // (the host stops counting applied passes here)
    }
}

// The pass's merges applied, a wave per slice (unless a list overflowed: then the pass is dropped
// whole and the host compacts what the earlier passes made), the pass's seed bits cleared for reuse
// (later passes: their seed bitmaps alternate), and the pass's totals for the host (workgroup 0).
__global__ __launch_bounds__(256) void sparse_apply_kernel(SparseParams q) {
    __shared__ uint32_t s_t[2][4];
    if (sp_gated(q)) return;
    const bool skip = *q.flags != 0u;
    const int lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (!skip) {
        const uint32_t nm = min(q.cnt_merges[w], q.slice);
        const uint32_t* ms = q.merges + 3ull * w * q.slice;
        for (uint32_t e = (uint32_t)lane; e < nm; e += 64u) {
            const uint32_t i = ms[3u * e], j = ms[3u * e + 1u];
            q.tok[i] = (uint16_t)ms[3u * e + 2u];
            atomicOr(&q.holes[j >> 5], 1u << (j & 31u));
            atomicAdd(&q.tile_cnt[j / kSparseTile], 1u);   // holes per compaction tile
        }
    }
    if (q.cnt_in && !skip) {   // (the first pass's bitmap is not reused; after an overflow the
                               // counts may be stale, and the next run's detect rewrites the bitmaps)
        const uint32_t ns = min(q.cnt_in[w], q.slice);
        const uint32_t* ss = q.seeds_in + (uint64_t)w * q.slice;
        for (uint32_t e = (uint32_t)lane; e < ns; e += 64u) {
            const uint32_t sd = ss[e];
            atomicAnd(&q.bits_in[sd >> 5], ~(1u << (sd & 31u)));
        }
    }
    if (skip || blockIdx.x != 0) return;
    uint32_t tm = 0, ts = 0;
    for (uint32_t k = threadIdx.x; k < q.nslices; k += 256u) {
        tm += min(q.cnt_merges[k], q.slice);
        ts += min(q.cnt_seeds[k], q.slice);
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        tm += (uint32_t)__shfl_xor((int)tm, d, 64);
        ts += (uint32_t)__shfl_xor((int)ts, d, 64);
    }
    if (lane == 0) {
        s_t[0][threadIdx.x >> 6] = tm;
        s_t[1][threadIdx.x >> 6] = ts;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        *q.nmerges = s_t[0][0] + s_t[0][1] + s_t[0][2] + s_t[0][3];
        *q.nseeds_out = s_t[1][0] + s_t[1][1] + s_t[1][2] + s_t[1][3];
    }
}

// Compaction of the hole layout in place.  The apply kernels counted the holes per tile of 8192
// positions; one workgroup scans the counts (a tile's output position is its first position less the
// holes before it; per-block sums over the counts cost more than that kernel).  A workgroup per
// kMoveGroup consecutive tiles (8192 positions a tile: 8-token groups, four per thread, consecutive
// lanes on consecutive groups), loads their input at once and marks it read, then per tile stages its
// tokens in LDS, waits until every earlier tile whose input its output range overlaps has marked its
// own (the output of tile T lies in [0, end of T's input): the one or two tiles its range falls in),
// and writes the range with 16-byte stores (2-byte ones at the two partial ends, which the
// neighbouring tiles share).  Small workgroup halves, many per CU (six waves per SIMD): the loads of
// the tiles in flight hide each other's latency.
// Progress (round 6): a workgroup's tiles come from a ticket (one atomic per
// workgroup), so every tile a workgroup waits for belongs to a lower ticket, i.e. to a workgroup
// that has started, loaded its tiles and marked them before any wait of its own; the lowest
// unfinished ticket waits for nobody.  No assumption on the order the hardware dispatches
// workgroups in, and none on other kernels sharing the device (round 5 relied on blockIdx order per
// XCD, and two such kernels on two streams could starve each other).  Four tiles per ticket keep the
// atomics (~11 ns each on one word, tools/atomic_probe.hip) at a quarter of round 4's one per tile.
constexpr int kCpThreads = 256;
constexpr uint64_t kMvRead = 1ull << 61;   // a tile's input is read (the list kernel's published counts use bit 62)
static_assert(kSparseTile == 32u * kCpThreads, "compaction tile");
static_assert(kSparseSampleBlocks == 64, "the detect gate sums the sample with one wave");

// The tiles' hole counts turned in place into the holes before each tile, and the total into
// *super_cnt: one workgroup, 16 consecutive counts per thread (four 16-byte loads, lanes on
// consecutive 64 bytes), rounds of 16384 tiles with the carry between them.
__global__ __launch_bounds__(1024) void sparse_tile_scan_kernel(SparseParams qa, const uint32_t* nseeds0) {
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_carry;
    if (sp_compact_skip(qa, nseeds0)) return;
    SparseParams q = qa;
    q.n = *qa.n_dev;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t ntiles = (q.n + kSparseTile - 1) / kSparseTile;
    const uint64_t nt16 = (ntiles + 15) & ~15ull;   // (the count array is padded: zeroed, 16-byte aligned)
    if (tid == 0) s_carry = 0u;
    __syncthreads();
    for (uint64_t r0 = 0; r0 < nt16; r0 += 16 * 1024) {
        const uint64_t t0 = r0 + 16ull * tid;
        uint32_t c[16];
        if (t0 < nt16) {
            const uint4* src = reinterpret_cast<const uint4*>(q.tile_cnt + t0);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 v = src[k];
                c[4 * k] = v.x; c[4 * k + 1] = v.y; c[4 * k + 2] = v.z; c[4 * k + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) c[k] = 0u;
        }
        uint32_t h = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) h += c[k];
        const uint32_t incl = wave_incl_scan(h, (int)lane);
        if (lane == 63) s_w[wave] = incl;
        __syncthreads();
        uint32_t before = s_carry, tot = 0;
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t v = s_w[k];
            before += k < wave ? v : 0u;
            tot += v;
        }
        before += incl - h;
        if (t0 < nt16) {
            uint32_t o[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                o[k] = before;
                before += c[k];
            }
            uint4* dst = reinterpret_cast<uint4*>(q.tile_cnt + t0);
#pragma unroll
            for (int k = 0; k < 4; ++k) dst[k] = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
        }
        __syncthreads();   // (s_w and s_carry read)
        if (tid == 0) s_carry += tot;
        __syncthreads();
    }
    if (tid == 0) *q.super_cnt = s_carry;
}

// A workgroup is two halves of kCpThreads threads; each half takes two consecutive tiles and loads
// both at once (twice the loads in flight per half at 6 waves per SIMD: selfval 0.699-0.710 ->
// 0.694 ms in round 5; four tiles per half spill).  The halves run the same steps between the
// workgroup's barriers; a half without a tile (the grid's last workgroup) only keeps step.
constexpr int kMoveTiles = 2;                    // tiles per half
// (Measured on selfval, round 6: one half per workgroup, 2 tiles per ticket, 0.737-0.754 ms; two,
// 0.715-0.722; three, 0.720-0.724.)
constexpr int kMoveHalves = 2;
constexpr int kMoveGroup = kMoveTiles * kMoveHalves;   // tiles per ticket
__global__ __launch_bounds__(kCpThreads * kMoveHalves) __attribute__((amdgpu_waves_per_eu(6)))
void sparse_move_kernel(SparseParams qa, const uint32_t* nseeds0) {
    // staged tokens, shifted by the output's offset in its 8-token group so that every output group
    // is one aligned 16-byte LDS word
    __shared__ __attribute__((aligned(16))) uint16_t s_out[kMoveHalves][kSparseTile + 8];
    __shared__ uint32_t s_wsum[kMoveHalves][4][kCpThreads / 64];
    __shared__ uint32_t s_tk, s_bad[kMoveHalves];
    if (sp_compact_skip(qa, nseeds0)) return;
    const int half = (int)threadIdx.x / kCpThreads;
    const int tid = (int)threadIdx.x % kCpThreads, lane = tid & 63, wave = tid >> 6;
    const uint64_t n = *qa.n_dev, ntiles = (n + kSparseTile - 1) / kSparseTile;
    if (threadIdx.x == 0) s_tk = atomicAdd(qa.super_cnt + 2, 1u);   // (zeroed with the run's counters)
    __syncthreads();
    const uint64_t G0 = (uint64_t)s_tk * kMoveGroup;
    if (G0 >= ntiles) return;   // (uniform: the grid is sized for the host's count, >= the device's)
    const uint64_t T0 = G0 + (uint64_t)half * kMoveTiles;
    // level j of tile t: 8-token group G = j * kCpThreads + tid
    uint32_t w[kMoveTiles][4][4], valid[kMoveTiles][4];
#pragma unroll
    for (int t = 0; t < kMoveTiles; ++t) {
        const uint64_t tile0 = (T0 + t) * kSparseTile;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t G = (uint32_t)j * kCpThreads + (uint32_t)tid;
            const uint64_t p = tile0 + 8ull * G;
            valid[t][j] = 0u;
            w[t][j][0] = w[t][j][1] = w[t][j][2] = w[t][j][3] = 0u;
            if (p < n) {
                const uint64_t left = n - p;
                valid[t][j] = ~(qa.holes[p >> 5] >> (8u * (G & 3u))) & (left >= 8 ? 0xFFu : ((1u << left) - 1u));
                if (left >= 8) {
                    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(qa.tok + p));
                    w[t][j][0] = v.x; w[t][j][1] = v.y; w[t][j][2] = v.z; w[t][j][3] = v.w;
                } else {   // (unrolled: a dynamic index would put w in scratch memory)
#pragma unroll
                    for (uint32_t k = 0; k < 7; ++k)
                        if (k < left) w[t][j][k >> 1] |= (uint32_t)qa.tok[p + k] << (16u * (k & 1u));
                }
            }
        }
    }
    // every tile of the workgroup marked read at once: a mark published only when the tile's turn
    // comes chains the workgroups (the first tile of workgroup b waits for the last one of
    // workgroup b - 1, which waits for its first ...: measured 30.8 ms on selfval)
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): every load of the workgroup's tiles
    __syncthreads();
    if (threadIdx.x < (uint32_t)kMoveGroup && G0 + threadIdx.x < ntiles) st_publish(qa.status + G0 + threadIdx.x, kMvRead);
#pragma unroll
    for (int t = 0; t < kMoveTiles; ++t) {
        const uint64_t T = T0 + t;
        const bool here = T < ntiles;   // (uniform per half; the halves keep step at every barrier)
        const uint64_t tile0 = T * kSparseTile;
        const uint32_t hb = here ? qa.tile_cnt[T] : 0u;   // holes before the tile (sparse_tile_scan_kernel)
        const uint32_t hnext = !here ? 0u : T + 1 < ntiles ? qa.tile_cnt[T + 1] : *qa.super_cnt;
        const uint64_t O = tile0 - hb;
        const uint32_t e = (uint32_t)(O & 7u);
        uint32_t cnt[4], incl[4];
        if (t) __syncthreads();   // (the previous tile's s_out and s_wsum read)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            cnt[j] = __popc(valid[t][j]);
            incl[j] = wave_incl_scan(cnt[j], lane);
            if (lane == 63) s_wsum[half][j][wave] = incl[j];
        }
        __syncthreads();
        uint32_t lbase = e;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t wb = 0, lt = 0;
#pragma unroll
            for (int k = 0; k < kCpThreads / 64; ++k) {
                const uint32_t v = s_wsum[half][j][k];
                wb += k < wave ? v : 0u;
                lt += v;
            }
            uint32_t o = lbase + wb + incl[j] - cnt[j];
            if (valid[t][j] == 0xFFu && (o & 1u) == 0u) {
                uint32_t* d = reinterpret_cast<uint32_t*>(s_out[half]) + (o >> 1);
                d[0] = w[t][j][0]; d[1] = w[t][j][1]; d[2] = w[t][j][2]; d[3] = w[t][j][3];
            } else {
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k) {
                    if ((valid[t][j] >> k) & 1u) s_out[half][o++] = (uint16_t)(w[t][j][k >> 1] >> (16u * (k & 1u)));
                }
            }
            lbase += lt;
        }
        const uint32_t ttot = lbase - e + ((qa.inject & kInjectSparseMove) ? 1u : 0u);   // (test hook)
        const uint64_t in_end = tile0 + kSparseTile < n ? tile0 + kSparseTile : n;
        // the tile's count against the scan's hole counts (the bitmap against the apply kernels'
        // counters): a tile whose counts disagree, or whose output would not lie within its own
        // input, flags error bit 4 and writes nothing
        const bool counts_ok = here && ttot == (in_end - tile0) - (hnext - hb) && hb <= tile0 && O + ttot <= in_end;
        if (tid == 0 && here && !counts_ok) flag_error(qa.ctl, qa.sticky, 4u);
        const bool moves = counts_ok && !(O == tile0 && ttot == in_end - tile0);   // (else in place already)
        if (tid == 0) s_bad[half] = 0u;
        __syncthreads();   // staged: every load of the tile done
        if (moves && wave == 0) {   // the earlier tiles whose input the output range overlaps (one or two)
            bool bad = false;
            const uint64_t ulast = ttot ? (O + ttot - 1) / kSparseTile : 0;
            const uint64_t uend = ulast + 1 < T ? ulast + 1 : T;
            for (uint64_t u = O / kSparseTile + (uint64_t)lane; u < uend; u += 64) {
                SpinClock clk;
                while ((st_read(qa.status + u) & kMvRead) == 0ull) {
                    if (clk.expired()) { bad = true; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            if (__ballot(bad) != 0ull && lane == 0) {
                flag_error(qa.ctl, qa.sticky, 1u);
                s_bad[half] = 1u;
            }
        }
        __syncthreads();
        // a wait that timed out (flagged): the input it waited for may be unread, so nothing is written
        if (!moves || s_bad[half]) continue;   // (uniform per half; no barrier before the next tile's)
        // output groups r = 0 .. nr - 1 (global tokens 8 (O / 8 + r) ..): whole ones with one 16-byte
        // store, the partial first and last token by token
        const uint32_t nr = (e + ttot + 7u) / 8u;
        uint16_t* dst = qa.tok + (O - e);
        for (uint32_t r = (uint32_t)tid; r < nr; r += kCpThreads) {
            const uint32_t b = 8u * r;
            if (b >= e && b + 8u <= e + ttot) {
                const v4u v = *reinterpret_cast<const v4u*>(s_out[half] + b);
                __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(dst + b));
            } else {
                for (uint32_t k = b; k < b + 8u; ++k)
                    if (k >= e && k < e + ttot) dst[k] = s_out[half][k];
            }
        }
    }
}

// Chunk offsets after the compaction (one wave per chunk): a chunk start (never a hole) moves left by
// the holes before it.  Block 0 also writes the total, to a word that may be the one the count came
// from (no other kernel here reads the count after this one starts).
__global__ __launch_bounds__(64) void sparse_coff_kernel(SparseParams q, const uint32_t* nseeds0) {
    const uint64_t c = blockIdx.x;
    const int lane = threadIdx.x;
    if (c >= q.nchunks || sp_compact_skip(q, nseeds0)) return;
    if (c == 0 && lane == 0) {
        const uint64_t total = *q.n_dev - *q.super_cnt;
        *q.total = total;
        q.coff_out[q.nchunks] = total;
    }
    const uint64_t p = q.coff_in[c];   // (< the count: every chunk holds a token)
    const uint64_t T = p / kSparseTile, wend = p >> 5;
    const uint32_t hb = q.tile_cnt[T];
    uint32_t cnt = 0;
    for (uint64_t wd = T * (kSparseTile / 32) + (uint64_t)lane; wd < wend; wd += 64) cnt += (uint32_t)__popc(~q.holes[wd]);
    if (lane == 0) cnt += (uint32_t)__popc(~q.holes[wend] & ((1u << (p & 31u)) - 1u));
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) cnt += (uint32_t)__shfl_xor((int)cnt, d, 64);
    if (lane == 0) q.coff_out[c] = T * kSparseTile - hb + cnt;
}

// Host check before any sparse launch: every list and bitmap set, positions in 32 bits.
static bool sparse_ok(const SparseParams& q) {
    return q.tok && q.n_dev && q.holes && q.bits_in && q.seeds_out && q.nseeds_out && q.bits_alt &&
           q.bits_out && q.merges && q.nmerges && q.flags && q.cap && q.hbuckets && q.coff_in && q.coff_out &&
           q.tile_cnt && q.super_cnt && q.status && q.sample && q.zero && q.n < (1ull << 32);
}
hipError_t launch_sparse_detect(const SparseParams& q, hipStream_t s) {
    if (!sparse_ok(q)) return hipErrorInvalidValue;
    // a lane per 32 positions; a grid of at most 8192 workgroups looping when the table is small
    // (each workgroup stages it), else 2048.  (selfval, 33 K workgroups of one round each: 145-148 us;
    // 8192: 134, 6144: 137, 12288: 135, 16384: 135, 4096: 143, 2048: 172, round 6, r06ac/r06ad.  A
    // workgroup per list workgroup's words, 16 rounds each, measured 240 us against 142.)
    const uint64_t nwords = (q.n + 31) / 32;
    uint64_t blocks = (nwords + 255) / 256;
    const bool lds = q.hbytes && q.hbytes <= kHashLdsMax;
    const uint64_t max_blocks = (lds && q.hbytes <= 4096) ? 8192 : 2048;
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(sparse_sample_kernel, dim3(kSparseSampleBlocks), dim3(1024), 0, s, q);
    const size_t smem = (lds ? ((q.hbytes + 15u) & ~15u) : 0u) + (q.nchunks <= kDetectCsLds ? 8 * q.nchunks : 0);
    if (lds)
        hipLaunchKernelGGL(sparse_detect_kernel<true>, dim3((unsigned)blocks), dim3(256), smem, s, q);
    else
        hipLaunchKernelGGL(sparse_detect_kernel<false>, dim3((unsigned)blocks), dim3(256), smem, s, q);
    return hipGetLastError();
}
hipError_t launch_sparse_list(const SparseParams& q, hipStream_t s) {
    if (!sparse_ok(q)) return hipErrorInvalidValue;
    // the host's count may exceed the device's: extra workgroups return
    const uint64_t nw = (q.n + 31) / 32, per = sp_list_words(nw);
    uint64_t g = (nw + per - 1) / per;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(sparse_list_kernel, dim3((unsigned)g), dim3(256), 0, s, q);
    return hipGetLastError();
}
hipError_t launch_sparse_pass(const SparseParams& q, hipStream_t s) {
    if (!sparse_ok(q) || !q.cnt_seeds || !q.cnt_merges || !q.slice || !q.nslices || q.nslices % 4 ||
        q.nslices > kSparseSlices || (uint64_t)q.slice * q.nslices > q.cap)
        return hipErrorInvalidValue;
    // a wave per slice, the same grid for both kernels (and every pass of the run)
    hipLaunchKernelGGL(sparse_region_kernel, dim3(q.nslices / 4u), dim3(256),
                       q.nchunks <= kDetectCsLds ? 8 * q.nchunks : 0, s, q);
    hipLaunchKernelGGL(sparse_apply_kernel, dim3(q.nslices / 4u), dim3(256), 0, s, q);
    return hipGetLastError();
}
hipError_t launch_sparse_compact(const SparseParams& q, const uint32_t* nseeds0, hipStream_t s) {
    if (!sparse_ok(q) || !q.total || !nseeds0 || !q.nchunks) return hipErrorInvalidValue;
    const uint64_t ntiles = (q.n + kSparseTile - 1) / kSparseTile;
    hipLaunchKernelGGL(sparse_tile_scan_kernel, dim3(1), dim3(1024), 0, s, q, nseeds0);
    hipLaunchKernelGGL(sparse_move_kernel, dim3((unsigned)((ntiles + kMoveGroup - 1) / kMoveGroup)),
                       dim3(kCpThreads * kMoveHalves), 0, s, q, nseeds0);
    hipLaunchKernelGGL(sparse_coff_kernel, dim3((unsigned)q.nchunks), dim3(64), 0, s, q, nseeds0);
    return hipGetLastError();
}

__global__ void noop_kernel() {}
hipError_t launch_noop(hipStream_t s) {
    hipLaunchKernelGGL(noop_kernel, dim3(1), dim3(64), 0, s);
    return hipGetLastError();
}

hipError_t launch_inject_error(uint32_t* ctl, uint32_t* sticky, hipStream_t s) {
    hipLaunchKernelGGL(inject_error_kernel, dim3(1), dim3(64), 0, s, ctl, sticky);
    return hipGetLastError();
}


}  // namespace blt
