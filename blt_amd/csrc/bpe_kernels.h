// Internal interface between the host library (blt_host.cpp) and the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace blt {

constexpr int kSub = 4;                       // sub-tiles per look-back tile
constexpr uint64_t kTilePos = 4 * 512 * 16;   // positions per look-back tile (kSub * threads * 16)
constexpr uint64_t kTilePosU16 = kTilePos;     // positions per look-back tile of the generic u16 pass
// (16384 measured and rejected: no VGPR spills, but twice the tiles and look-backs; f2 chain
// 0.672 -> 0.804 ms, selfval 1.39 -> 1.77, multi 0.537 -> 0.575; profiles/r04_shift16_ab.txt)
constexpr uint64_t kTilePosTok = 32768;        // tokens per look-back tile of the u16 scan kernel (32 wave ranges)
constexpr uint64_t kTokRange = 1024;           // tokens per wave range (one chunk-map word each)
constexpr uint64_t kTilePosBytes = 32768;      // positions per look-back tile of the byte-input pass
constexpr uint64_t kMinChunkBytes = 4096;      // byte pass needs chunk_size >= positions per wave range
constexpr uint64_t kCtlBytes = 64;            // control block ahead of the status words
constexpr uint32_t kCtlLeft = 15;             // ctl word: workgroups of a single-pass launch that have left
constexpr uint32_t kCtlTickAlt = 12;          // ctl word: the ticket of odd chained u16 scan passes
constexpr uint32_t kCtlCover = 14;            // ctl word: status words [0, ctl[14]) are known zero (set by
                                              // blt_bpe_workspace_reset and by a single-pass launch's self-reset);
                                              // a launch told its workspace is zeroed checks its tiles against it

// Parameters of one merge pass over a whole buffer of positions.
struct PassParams {
    const void* in;            // uint8_t bytes (pass 1) or uint16_t tokens (later passes)
    uint64_t n;                // number of positions
    uint64_t cs;               // chunk size in positions (pass 1), or 0 to use cstart
    const uint64_t* cstart;    // cs == 0: chunk start positions [0, nchunks)
    uint64_t nchunks;
    void* out;                 // big-endian u16 bytes, or native u16 tokens
    uint64_t* chunk_off;       // optional [nchunks + 1]: output token index of each chunk start
    uint64_t* status;          // [ntiles] look-back status words, zeroed before the launch
    uint32_t* ctl;             // [0] tile ticket, [1] error flags, [2..15] first-error record; zeroed
    uint64_t out_cap;          // bytes writable at out
    uint64_t* total;           // number of output tokens
    uint32_t ntiles;
    uint32_t sentinel;         // dense table: "absent" value; > 0xFFFF = every byte pair present
    const uint16_t* dense;     // dense byte-pair table (65536 entries, swizzled layout).  General
                               // kernel: native values, sentinel where absent.  Byte-pass kernel:
                               // self-token table (absent (a, b) -> a) in the output byte order
    const uint2* hbuckets;     // general map (u16 passes): 2-choice cuckoo table of one-slot
                               // buckets [key, val]; key = the pair's u16 words as stored (big-endian
                               // tokens), BE(a) | BE(b) << 16; val = BE(v) | 1 << 31 | live << 30 (live:
                               // v is a component of some key); empty buckets hold a key not in the
                               // map and val 0
    uint32_t hmul1, hmul2;     // bucket of key: dot2(key, hmul) >> hshift (u16 halves), two choices
    uint32_t hshift;
    uint32_t hbytes;           // table bytes (u16 passes stage the table in LDS when it fits)
    uint32_t hone;             // the table is one-probe: every key sits in bucket dot2(key, hmul1) >> hshift
                               // (hmul2 == hmul1, so two-probe readers stay correct)
    const uint64_t* n_dev;     // u16 passes: the token count written by the previous pass (on device)
    uint32_t* done;            // u16 passes: set to pass_id by the pass after which the next merges
                               // nothing (it merged nothing, or none of its merges made a key
                               // component); later passes return at once
    uint32_t pass_id;          // u16 passes: 1, 2, ... (pass k writes totals and chunk offsets [k & 1])
    uint64_t* cmap;            // u16 scan kernel: chunk-map word per wave range of kTokRange tokens
    uint64_t* cmap_next;       // u16 scan kernel (nullable): the next pass's chunk map, built from this
                               // pass's chunk offsets as it writes them (zeroed before this pass)
    uint64_t* cmap_zero;       // u16 scan kernel (nullable): the map the pass after next builds, zeroed here
    uint64_t* status_zero;     // u16 scan kernel (nullable): the next pass's status words (the other of two
                               // arrays), zeroed here with its ticket word ctl[tick ^ kCtlTickAlt]
    uint32_t tick;             // ctl word of the tile tickets: 0, or kCtlTickAlt for odd chained u16 passes
    uint64_t cs_magic;         // cs > 0: floor((2^64 - 1) / cs), for x / cs by a high multiply
    uint32_t cs_tiles;         // cs / kTilePosBytes when cs is a whole number of byte-pass tiles
                               // (below 2^31), else 0
    uint32_t cs_tiles_magic;   // floor((2^32 - 1) / cs_tiles) (cs_tiles > 1)
    uint32_t allm;             // byte pass: every byte pair is a merge (the entry's test is skipped)
    uint32_t mark;             // byte pass, mode 2: BE pattern (mark | mark << 16) of the high byte that
                               // marks a merge valued its own first byte
    uint32_t* sticky;          // the handle's pinned host error word (nullable): set to 1 with the
                               // error bits in ctl[1], so the handle's next call fails
    uint32_t* fin_gate;        // finish kernels: the longest chunk's tokens (capped), from the gate kernel
    uint32_t ws_check;         // single-pass byte kernels launched without a memset (BLT_ENCODE_WORKSPACE_ZEROED):
                               // refuse (error bit 32, no output) when ntiles > ctl[kCtlCover]
    uint32_t* fused_fail;      // fused passes 1 + 2: set to 1 when a wave range's halo holds no
                               // restart (the host then runs the two-kernel chain instead)
    uint64_t* debug;           // optional [ntiles * 8] per-tile record (tests only): [4T..]: O,
                               // C|how, counts, carry-outs; byte pass [4 ntiles + 4T..]: s_memtime at
                               // the iteration start, after the first and second barrier; spins
    uint32_t inject;           // test hook (kInject*): a count broken on purpose, 0 in production
};
// Test hook (blt_debug_set_inject): a kernel breaks one of its counts on purpose, to show that its
// invariant checks turn the count into a flagged error (BLT_E_IO) and no store lands outside the
// range the count should have given.  Finish kernel: the first pass's count; u16 scan: a tile's
// count; sparse move: a tile's count.
constexpr uint32_t kInjectFinish = 1u, kInjectScanTok = 2u, kInjectSparseMove = 4u;

// Generic pass: byte input with the dense LDS table (maps the byte pass cannot take), or BE u16
// tokens with the bucket table (p.hbuckets) for the later passes of a general map; output BE.
hipError_t launch_merge_pass(const PassParams& p, int input_u16, int big_endian, int device, hipStream_t s);
// Byte-input pass (segment kernel, seg::scan_bytes_kernel), big-endian output: p.cs >=
// kMinChunkBytes; tiles of kTilePosBytes positions.  mode: 0 every byte-pair merge value is >= 256,
// so an entry's high byte tells a merge; 1 an entry that differs from the token of a is a merge; 2
// as 1 with merges valued their own first byte marked (p.mark).  live (modes 1 and 2): the first
// pass of a general map whose keys are byte pairs; it sets *p.done = kDoneBytePass when it made no
// token below 256.
hipError_t launch_scan_bytes(const PassParams& p, int mode, int live, int device, hipStream_t s);
// done word value of a byte pass after which nothing merges (u16 pass k writes k)
constexpr uint32_t kDoneBytePass = 0x80000000u;
// u16 pass of a general map on the scan kernel (seg::scan_tokens_kernel), in place (p.in may equal
// p.out): when map_ready is 0, the chunk map of p.cstart into p.cmap first (and the status words and
// ticket zeroed); with map_ready the previous scan pass built p.cmap and reset its status words and
// ticket itself.  Needs every chunk but the last to hold at least kTokRange tokens.
hipError_t launch_scan_tokens(const PassParams& p, int map_ready, int device, hipStream_t s);
// Passes 1 and 2 of a general map in one kernel (seg::scan_tokens_kernel<kHash, true>): bytes in,
// the second pass's big-endian tokens out, for maps whose bucket table fits in LDS and chunk sizes
// >= kMinChunkBytes.  A wave range takes the first pass's carry-in from the 64 bytes before it
// (a greedy pass restarts after every pair it does not merge); the second pass's carries and every
// offset go through the u16 scan's look-back.  Writes p.total, p.chunk_off and p.done as u16 pass
// p.pass_id (1), or sets *p.fused_fail.
hipError_t launch_scan_fused(const PassParams& p, int device, hipStream_t s);
// The rest of a general map's chain from u16 pass p.pass_id on, per group of chunks in LDS
// (finish_gate_kernel, finish_chunks_kernel): in place in p.out (= p.in), chunk starts from p.cstart
// (the previous pass's offsets), status words at p.status (one per chunk), ticket p.ctl[0]; writes
// p.chunk_off, p.total and p.done = p.pass_id, or nothing when the longest chunk does not fit in LDS
// (the gate word *p.fin_gate, the longest chunk, must be zero before the launch).
hipError_t launch_finish(const PassParams& p, int device, hipStream_t s);
constexpr uint64_t kFinCapTokens = 16384;      // tokens of a group in LDS (finish_chunks_kernel)
constexpr uint32_t kFinMaxGroupChunks = 1024;  // chunks per group
hipError_t launch_basic_expand(const uint8_t* in, uint64_t n, uint8_t* out, hipStream_t s);
// The end of a general map's chain enqueued up to its known depth: the final pass (the done word's,
// else k_last) gives *tot_final and, when it wrote off1, the caller's chunk offsets.
hipError_t launch_chain_final(const uint64_t* tot, const uint32_t* done, const uint64_t* off1, uint64_t* chunk_off,
                              uint64_t nchunks, uint32_t k_last, uint64_t* tot_final, hipStream_t s);
// Sparse passes of a cyclic general map (round 4): once a chain's passes merge almost nothing, the
// tokens stay in place and consumed positions are marked in a hole bitmap; each pass runs only the
// maximal runs of mergeable pairs around the previous pass's new tokens, and one compaction writes the
// result.  Positions below 2^31.
struct SparseParams {
    uint16_t* tok;              // tokens as stored (big-endian u16), positions [0, n), in place
    uint64_t n;                 // an upper bound of the token count (grid sizes)
    const uint64_t* n_dev;      // the token count, read by every kernel on the device
    const uint64_t* gate;       // nonzero: the chain is done or must fall back; every kernel returns
    const uint32_t* cond;       // compaction kernels: run only when *cond == 0 (null: always)
    uint32_t* holes;            // bit p: position p was consumed by a merge (n bits)
    uint32_t* seeds_in;         // this pass's seeds (positions), bitmap bits_in: the first pass's a
                                // flat list of *nseeds_in, later passes' per-wave slices (cnt_in)
    uint32_t* nseeds_in;
    const uint32_t* cnt_in;     // per slice: seeds in it (null: the flat list)
    uint32_t* bits_in;
    uint32_t* seeds_out;        // the next pass's seeds: live tokens this pass made
    uint32_t* nseeds_out;
    uint32_t* bits_out;
    uint32_t* bits_alt;         // the later passes' other seed bitmap (the detect kernel zeroes it)
    uint32_t first_pass;        // 1: the first pass (an overflow leaves everything untouched)
    uint32_t* merges;           // (position, consumed position, value) per merge of this pass
    uint32_t* nmerges;          // totals of the pass (the apply kernel; cap + 1: a slice overflowed)
    uint32_t* cnt_seeds;        // per slice: next seeds this pass made (the region kernel)
    uint32_t* cnt_merges;       // per slice: merges this pass made
    uint32_t slice;             // entries per slice: the region kernel's wave w appends to entries
    uint32_t nslices;           // [w slice, (w + 1) slice) of seeds_out and merges, no atomics
    uint32_t* flags;            // [0]: a list overflowed (this pass is not applied)
    uint32_t cap;               // entries of each list
    const uint2* hbuckets;      // the map's bucket table (as PassParams)
    uint32_t hmul1, hmul2, hshift;
    uint32_t hbytes, hone;      // table bytes (staged in LDS by the detect kernel up to kHashLdsMax), one-probe table
    // compaction
    const uint64_t* coff_in;    // chunk starts (positions of the hole layout), [nchunks]
    uint64_t* coff_out;         // chunk offsets after compaction, [nchunks + 1]
    uint64_t nchunks;
    uint64_t* total;            // tokens after compaction (may be the word n_dev points to: written last)
    uint32_t* tile_cnt;         // per compaction tile: holes in it (apply kernels), then holes before it (scan)
    uint32_t* super_cnt;        // one word: the holes in all (scan)
    uint64_t* status;           // per compaction tile: the list kernel's seed counts, then the move's
                                // read marks (zeroed)
    uint32_t* ctl;              // the chain's control block (error flags)
    uint32_t* sticky;
    uint32_t* sample;           // detect's gate: mergeable pairs per sampled block (kSparseSampleBlocks
                                // words, written whole by the sample kernel)
    uint4* zero;                // the run's counters, tile counts and status words: zeroed by the
    uint32_t zero16;            // sample kernel (16-byte units), ahead of every other sparse kernel
    uint32_t inject;            // test hook (kInjectSparseMove), 0 in production
};
constexpr uint64_t kSparseTile = 8192;    // positions per compaction tile
// Region / apply kernels: 256-thread workgroups, one list slice per wave (at most kSparseSlices)
constexpr uint32_t kSparseSlices = 4096;
// Positions the detect gate samples: kSparseSampleBlocks evenly spaced runs of 8192 positions.
constexpr uint32_t kSparseSampleBlocks = 64;
constexpr uint32_t kSparseSample = kSparseSampleBlocks * 8192u;
// detect: the first pass's seeds (every mergeable pair's first position) into seeds_in / bits_in.
// A sampling kernel runs first (it also zeroes the run's counters: no memset), and detect leaves the
// run not taken (flags 3, no bitmaps) when the sample predicts more than half the lists' capacity of
// seeds: a dense cyclic map goes on with the full passes for the cost of a few empty launches
// (ADVICE r4).
hipError_t launch_sparse_detect(const SparseParams& q, hipStream_t s);
// the first pass's seed list from the detect kernel's bitmap (q.seeds_out, q.nseeds_out)
hipError_t launch_sparse_list(const SparseParams& q, hipStream_t s);
// one pass: regions (reads only; merges and new seeds into lists), then the merges applied and the
// input seeds' bits cleared
hipError_t launch_sparse_pass(const SparseParams& q, hipStream_t s);
// the hole layout compacted in place: tokens, chunk offsets, total (nseeds0: the detect kernel's
// seed count; nothing runs when it overflowed the lists)
hipError_t launch_sparse_compact(const SparseParams& q, const uint32_t* nseeds0, hipStream_t s);
// An empty kernel: the first launch of any kernel loads the library's code object on the device
// (the CLI's start-up does it on its helper thread, beside the input's mmap).
hipError_t launch_noop(hipStream_t s);
// Test hook: runs the kernels' error path once (ctl nullable, sticky the handle's error word).
hipError_t launch_inject_error(uint32_t* ctl, uint32_t* sticky, hipStream_t s);

// Dense-table layout shared with the host: entry for byte pair (a, b).
inline uint32_t dense_index(uint32_t a, uint32_t b) { return (a << 8) | (b ^ ((a << 1) & 0xFEu)); }

// Self-token table of the byte pass: rows of kSelfRow u16 entries (256 used), entry (a, b) at
// a * kSelfRow + b.  The 2-entry pad per row skews rows across the LDS banks: the dword of (a, b)
// is 129 a + b / 2, its bank (a + b / 2) mod 32, so lanes reading pairs with the same second byte
// (English text) spread over the banks; the byte address 516 a + 2 b + base is one v_dot2_u32_u16.
constexpr uint32_t kSelfRow = 258;
constexpr uint32_t kSelfEntries = 256 * kSelfRow;
inline uint32_t self_index(uint32_t a, uint32_t b) { return a * kSelfRow + b; }

// Bucket of a general-map key (must match bucket_get in bpe_kernels.hip): the top bits of
// v_dot2_u32_u16(key, mul) = lo(key) lo(mul) + hi(key) hi(mul) mod 2^32.
inline uint32_t bucket_of(uint32_t key, uint32_t mul, uint32_t shift) {
    return (uint32_t)((key & 0xFFFFu) * (mul & 0xFFFFu) + (key >> 16) * (mul >> 16)) >> shift;
}
// Largest general-map table staged in LDS (bytes); larger tables are read from global memory (L2).
constexpr uint32_t kHashLdsMax = 48u << 10;

}  // namespace blt
