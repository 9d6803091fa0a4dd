// Synthetic workload generators for the BPE merge-scan benchmarks and parity tests.
//
// Not part of the tokenizer itself: these produce the seeded inputs that SURVEY.md §8(d) names
// (cfg1 random bytes, cfg2/cfg3/cfg4 synthetic English-like text, cfg5 random bytes) and the
// adjacent-pair histogram used to rank merges.  Every stream is generated in independent
// 1 MiB blocks (block j seeded from (seed, j) through splitmix64), so any byte range of an
// arbitrarily long stream can be produced on its own — each rank of a multi-GPU run makes
// only its own shard, and OpenMP fills blocks in parallel.  Python tests call the same code
// through ctypes, so the bytes are identical everywhere.
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>

#define SYNTH_BLOCK ((size_t)1 << 20)

static inline uint64_t sm64_next(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static inline uint64_t block_state(uint64_t seed, uint64_t block) {
    uint64_t s = seed * 0xD1B54A32D192ED03ULL + block * 0x9E3779B97F4A7C15ULL + 0x632BE59BD9B4E019ULL;
    (void)sm64_next(&s);
    return s;
}

// English letter frequencies (per 99 999), a..z.
static const uint32_t kFreq[26] = {8167, 1492, 2782, 4253, 12702, 2228, 2015, 6094, 6966, 153,
                                   772,  4025, 2406, 6749, 7507,  1929, 95,   5987, 6327, 9056,
                                   2758, 978,  2360, 150,  1974,  74};

static uint32_t g_cdf[26];
static int g_cdf_ready = 0;

static void init_cdf(void) {
    if (g_cdf_ready) return;
    uint32_t acc = 0;
    for (int i = 0; i < 26; ++i) { acc += kFreq[i]; g_cdf[i] = acc; }  // acc ends at 99 999
    g_cdf_ready = 1;
}

static inline uint8_t draw_letter(uint64_t *s) {
    uint32_t r = (uint32_t)(sm64_next(s) % 99999u);
    int lo = 0, hi = 25;
    while (lo < hi) { int mid = (lo + hi) >> 1; if (r < g_cdf[mid]) hi = mid; else lo = mid + 1; }
    return (uint8_t)('a' + lo);
}

// One text block: words of geometric length (continue with p = 0.78, capped at 12) over a-z with
// English letter frequencies, separated by ' ' or, with probability 1/12, '\n'.  The block is
// cut at exactly `len` bytes (the last word may be truncated).
static void text_block(uint8_t *dst, size_t len, uint64_t seed, uint64_t block) {
    uint64_t s = block_state(seed, block);
    const uint64_t p_cont = (uint64_t)(0.78 * (double)(1u << 24));
    size_t pos = 0;
    while (pos < len) {
        int wl = 1;
        while (wl < 12 && (sm64_next(&s) >> 40) < p_cont) ++wl;
        for (int i = 0; i < wl && pos < len; ++i) dst[pos++] = draw_letter(&s);
        if (pos < len) dst[pos++] = (sm64_next(&s) % 12u == 0) ? '\n' : ' ';
    }
}

static void random_block(uint8_t *dst, size_t len, uint64_t seed, uint64_t block) {
    uint64_t s = block_state(seed ^ 0xA5A5A5A5A5A5A5A5ULL, block);
    size_t pos = 0;
    while (pos + 8 <= len) { uint64_t r = sm64_next(&s); memcpy(dst + pos, &r, 8); pos += 8; }
    if (pos < len) { uint64_t r = sm64_next(&s); memcpy(dst + pos, &r, len - pos); }
}

typedef void (*block_fn)(uint8_t *, size_t, uint64_t, uint64_t);

// Fills dst with bytes [offset, offset + n) of the stream.
static void fill_range(block_fn fn, uint8_t *dst, uint64_t offset, size_t n, uint64_t seed) {
    if (n == 0) return;
    uint64_t first = offset / SYNTH_BLOCK, last = (offset + n - 1) / SYNTH_BLOCK;
    long long nb = (long long)(last - first + 1);
#pragma omp parallel for schedule(dynamic, 4)
    for (long long i = 0; i < nb; ++i) {
        uint64_t b = first + (uint64_t)i;
        uint64_t bstart = b * SYNTH_BLOCK;
        uint64_t lo = bstart > offset ? bstart : offset;
        uint64_t hi = bstart + SYNTH_BLOCK < offset + n ? bstart + SYNTH_BLOCK : offset + n;
        if (lo == bstart && hi == bstart + SYNTH_BLOCK) {
            fn(dst + (lo - offset), SYNTH_BLOCK, seed, b);
        } else {
            uint8_t *tmp = (uint8_t *)malloc(SYNTH_BLOCK);
            fn(tmp, SYNTH_BLOCK, seed, b);
            memcpy(dst + (lo - offset), tmp + (lo - bstart), hi - lo);
            free(tmp);
        }
    }
}

void blt_synth_text(uint8_t *dst, uint64_t offset, size_t n, uint64_t seed) {
    init_cdf();
    fill_range(text_block, dst, offset, n, seed);
}

void blt_synth_random(uint8_t *dst, uint64_t offset, size_t n, uint64_t seed) {
    fill_range(random_block, dst, offset, n, seed);
}

// counts[a * 256 + b] += number of i < n - 1 with (p[i], p[i + 1]) == (a, b).
void blt_synth_pair_counts(const uint8_t *p, size_t n, uint64_t *counts) {
    if (n < 2) return;
    const size_t step = (size_t)1 << 22;
    long long nparts = (long long)((n - 1 + step - 1) / step);
#pragma omp parallel
    {
        uint64_t *local = (uint64_t *)calloc(65536, sizeof(uint64_t));
#pragma omp for schedule(static)
        for (long long k = 0; k < nparts; ++k) {
            size_t lo = (size_t)k * step, hi = lo + step < n - 1 ? lo + step : n - 1;
            for (size_t i = lo; i < hi; ++i) local[((unsigned)p[i] << 8) | p[i + 1]]++;
        }
#pragma omp critical
        for (int i = 0; i < 65536; ++i) counts[i] += local[i];
        free(local);
    }
}
