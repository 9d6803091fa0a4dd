// =====================================================================================
//  ORACLE — TEST INFRASTRUCTURE ONLY.  NOT PART OF THE PRODUCT PATH.
//
//  A plain-C restatement of the reference's CPU path for the BPE merge scan
//  (jtrefon/blt @ /root/reference).  Only tests/, __graft_entry__.smoke() and bench.py's
//  cpu_baseline leg may load this library, and only as the checker / the CPU baseline;
//  the GPU product (blt_amd/, libblt_bpe.so) never links or calls it.
//
//  Parity status: the reference is Rust and no Rust toolchain exists in this image, so the
//  reference cannot be run here.  This restatement is pinned by the reference's own
//  known-answer tests (blt_core/src/tokenizer.rs:170-291, config_loader.rs:61-202,
//  chunking.rs:96-113, utils.rs:51-71, tests/cli.rs:20-214), transcribed as data into
//  tests/golden/reference_kats.json and checked by tests/test_oracle_kats.py.
//
//  Every function cites the reference file:line it follows.
// =====================================================================================
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define ORC_OK 0
#define ORC_NOT_FOUND 1     // io::ErrorKind::NotFound
#define ORC_INVALID_DATA 2  // io::ErrorKind::InvalidData
#define ORC_OTHER_IO 3      // any other io::Error
#define ORC_NOSPACE 4       // caller's arrays too small (oracle plumbing, not a reference error)

static void set_msg(char *msg, size_t cap, const char *fmt, const char *a, const char *b) {
    if (!msg || cap == 0) return;
    snprintf(msg, cap, fmt, a, b);
}

// ---------------------------------------------------------------------------------------
// UTF-8 helpers: Rust's BufRead::lines() rejects invalid UTF-8 with InvalidData
// ("stream did not contain valid UTF-8"), and str::split_whitespace() splits on Unicode
// White_Space.
// ---------------------------------------------------------------------------------------
// Decodes one code point at s[0..n); returns its byte length, or 0 if invalid.
static int utf8_decode(const unsigned char *s, size_t n, uint32_t *cp) {
    if (n == 0) return 0;
    unsigned c = s[0];
    if (c < 0x80) { *cp = c; return 1; }
    int len; uint32_t v; uint32_t min;
    if ((c & 0xE0) == 0xC0) { len = 2; v = c & 0x1F; min = 0x80; }
    else if ((c & 0xF0) == 0xE0) { len = 3; v = c & 0x0F; min = 0x800; }
    else if ((c & 0xF8) == 0xF0) { len = 4; v = c & 0x07; min = 0x10000; }
    else return 0;
    if ((size_t)len > n) return 0;
    for (int i = 1; i < len; ++i) {
        if ((s[i] & 0xC0) != 0x80) return 0;
        v = (v << 6) | (s[i] & 0x3F);
    }
    if (v < min || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) return 0;
    *cp = v;
    return len;
}

static int utf8_valid(const unsigned char *s, size_t n) {
    size_t i = 0; uint32_t cp;
    while (i < n) { int l = utf8_decode(s + i, n - i, &cp); if (!l) return 0; i += (size_t)l; }
    return 1;
}

// char::is_whitespace (Unicode White_Space property).
static int uni_space(uint32_t c) {
    return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
           (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F ||
           c == 0x205F || c == 0x3000;
}

// Splits a valid UTF-8 line like str::split_whitespace; returns number of fields, fills up to
// `maxf` (start, len) pairs.
static int split_ws(const unsigned char *s, size_t n, size_t *st, size_t *ln, int maxf) {
    int nf = 0; size_t i = 0; int in_field = 0; size_t fs = 0;
    while (i < n) {
        uint32_t cp; int l = utf8_decode(s + i, n - i, &cp);
        if (l == 0) l = 1;  // unreachable: line already validated
        if (uni_space(cp)) {
            if (in_field) { if (nf < maxf) { st[nf] = fs; ln[nf] = i - fs; } nf++; in_field = 0; }
        } else if (!in_field) { in_field = 1; fs = i; }
        i += (size_t)l;
    }
    if (in_field) { if (nf < maxf) { st[nf] = fs; ln[nf] = n - fs; } nf++; }
    return nf;
}

// <u8 as FromStr>::from_str (core::num, radix 10): optional '+', ASCII digits only.
// For each char the digit is checked before the multiply's overflow is reported.
// Returns 0 ok, 1 InvalidDigit, 2 PosOverflow, 3 Empty.
static int parse_u8(const unsigned char *s, size_t n, unsigned *out) {
    if (n == 0) return 3;
    size_t i = 0;
    if (s[0] == '+' || s[0] == '-') {
        if (n == 1) return 1;
        if (s[0] == '+') i = 1;  // '-' stays and fails as an invalid digit (unsigned type)
    }
    unsigned r = 0;
    for (; i < n; ++i) {
        int mul_ok = r * 10u <= 255u;
        if (s[i] < '0' || s[i] > '9') return 1;
        if (!mul_ok) return 2;
        r = r * 10u + (unsigned)(s[i] - '0');
        if (r > 255u) return 2;
    }
    *out = r;
    return 0;
}

static const char *pie_text(int kind) {
    switch (kind) {
        case 1: return "invalid digit found in string";
        case 2: return "number too large to fit in target type";
        default: return "cannot parse integer from empty string";
    }
}

// ---------------------------------------------------------------------------------------
// load_bpe_merges_from_path — blt_core/src/config_loader.rs:14-46.
//   line i (valid, 0-based) -> (u8, u8) => 256 + i, u16 counter wrapping (release build, no
//   overflow-checks in /root/reference/Cargo.toml); duplicates overwrite, the counter still
//   advances (:39-40); skip lines that are empty or start with '#' (:22); exactly two
//   whitespace-separated fields else InvalidData (:41-43).
// Output: the final map as arrays sorted by key.  The message matches the reference's
// io::Error Display text.
// ---------------------------------------------------------------------------------------
int oracle_load_merges(const char *path, uint16_t *ka, uint16_t *kb, uint16_t *kv, size_t cap,
                       size_t *n_out, char *msg, size_t msgcap) {
    *n_out = 0;
    FILE *f = fopen(path, "rb");
    if (!f) {
        int e = errno;
        char buf[64]; snprintf(buf, sizeof buf, "%d", e);
        set_msg(msg, msgcap, "%s (os error %s)", strerror(e), buf);
        return e == ENOENT ? ORC_NOT_FOUND : ORC_OTHER_IO;
    }
    size_t size = 0, capb = 1 << 16;
    unsigned char *data = (unsigned char *)malloc(capb);
    for (;;) {
        if (size == capb) { capb *= 2; data = (unsigned char *)realloc(data, capb); }
        size_t r = fread(data + size, 1, capb - size, f);
        if (r == 0) {
            if (ferror(f)) {
                int e = errno ? errno : EIO;
                char buf[64]; snprintf(buf, sizeof buf, "%d", e);
                set_msg(msg, msgcap, "%s (os error %s)", strerror(e), buf);
                fclose(f); free(data);
                return ORC_OTHER_IO;
            }
            break;
        }
        size += r;
    }
    fclose(f);

    // value table indexed by key a*256+b; -1 = absent
    int32_t *val = (int32_t *)malloc(65536 * sizeof(int32_t));
    for (int i = 0; i < 65536; ++i) val[i] = -1;
    uint16_t vocab = 256;
    size_t pos = 0;
    int rc = ORC_OK;
    char *linebuf = NULL; size_t linecap = 0;
    while (pos < size) {
        // BufRead::read_line: up to and including '\n'; lines() pops "\n" then a "\r".
        size_t e = pos;
        while (e < size && data[e] != '\n') ++e;
        size_t len = e - pos;
        int had_nl = e < size;
        const unsigned char *line = data + pos;
        size_t next = had_nl ? e + 1 : e;
        if (!utf8_valid(line, len + (had_nl ? 1 : 0))) {
            set_msg(msg, msgcap, "%s%s", "stream did not contain valid UTF-8", "");
            rc = ORC_INVALID_DATA; break;
        }
        if (had_nl && len > 0 && line[len - 1] == '\r') len -= 1;
        pos = next;
        if (len == 0 || line[0] == '#') continue;
        if (len + 1 > linecap) { linecap = len + 1; linebuf = (char *)realloc(linebuf, linecap); }
        memcpy(linebuf, line, len); linebuf[len] = 0;
        size_t st[3], ln[3];
        int nf = split_ws(line, len, st, ln, 3);
        if (nf != 2) {
            set_msg(msg, msgcap,
                    "Invalid merge rule format in line: '%s'. Expected two numbers separated by space.%s",
                    linebuf, "");
            rc = ORC_INVALID_DATA; break;
        }
        unsigned b1, b2; int k;
        if ((k = parse_u8(line + st[0], ln[0], &b1)) != 0) {
            char tmp[96]; snprintf(tmp, sizeof tmp, "%s", pie_text(k));
            set_msg(msg, msgcap, "Failed to parse first byte value: %s in line '%s'", tmp, linebuf);
            rc = ORC_INVALID_DATA; break;
        }
        if ((k = parse_u8(line + st[1], ln[1], &b2)) != 0) {
            char tmp[96]; snprintf(tmp, sizeof tmp, "%s", pie_text(k));
            set_msg(msg, msgcap, "Failed to parse second byte value: %s in line '%s'", tmp, linebuf);
            rc = ORC_INVALID_DATA; break;
        }
        val[(b1 << 8) | b2] = vocab;
        vocab = (uint16_t)(vocab + 1);
    }
    free(linebuf);
    free(data);
    if (rc == ORC_OK) {
        size_t n = 0;
        for (int i = 0; i < 65536; ++i) if (val[i] >= 0) ++n;
        *n_out = n;
        if (n > cap) { free(val); return ORC_NOSPACE; }
        size_t j = 0;
        for (int i = 0; i < 65536; ++i)
            if (val[i] >= 0) { ka[j] = (uint16_t)(i >> 8); kb[j] = (uint16_t)(i & 255); kv[j] = (uint16_t)val[i]; ++j; }
    }
    free(val);
    return rc;
}

// ---------------------------------------------------------------------------------------
// BpeMerges = HashMap<(u16, u16), u16> — blt_core/src/lib.rs:75.  Open addressing on the
// packed key; built from pairs in order so that a later duplicate overwrites (collect()).
// ---------------------------------------------------------------------------------------
typedef struct {
    uint64_t *slots;  // bit 63 occupied | value << 32 | key
    uint64_t mask;
    size_t count;
} omap;

static inline uint64_t hash32(uint32_t k) {
    uint64_t x = k * 0x9E3779B97F4A7C15ULL;
    return x ^ (x >> 29);
}

omap *oracle_map_new(const uint16_t *a, const uint16_t *b, const uint16_t *v, size_t n) {
    omap *m = (omap *)calloc(1, sizeof(omap));
    uint64_t capn = 16;
    while (capn < 2 * (uint64_t)n + 2) capn <<= 1;
    m->slots = (uint64_t *)calloc(capn, sizeof(uint64_t));
    m->mask = capn - 1;
    for (size_t i = 0; i < n; ++i) {
        uint32_t key = ((uint32_t)a[i] << 16) | b[i];
        uint64_t h = hash32(key) & m->mask;
        for (;;) {
            uint64_t s = m->slots[h];
            if (!(s >> 63)) { m->slots[h] = (1ULL << 63) | ((uint64_t)v[i] << 32) | key; m->count++; break; }
            if ((uint32_t)s == key) { m->slots[h] = (1ULL << 63) | ((uint64_t)v[i] << 32) | key; break; }
            h = (h + 1) & m->mask;
        }
    }
    return m;
}

void oracle_map_free(omap *m) {
    if (!m) return;
    free(m->slots);
    free(m);
}

static inline int map_get(const omap *m, uint16_t x, uint16_t y, uint16_t *out) {
    uint32_t key = ((uint32_t)x << 16) | y;
    uint64_t h = hash32(key) & m->mask;
    for (;;) {
        uint64_t s = m->slots[h];
        if (!(s >> 63)) return 0;
        if ((uint32_t)s == key) { *out = (uint16_t)(s >> 32); return 1; }
        h = (h + 1) & m->mask;
    }
}

// ---------------------------------------------------------------------------------------
// BpeStrategy::process_chunk — blt_core/src/tokenizer.rs:56-93.
//   empty -> empty (:57-59); widen to u16 (:61); greedy left-to-right passes, a mapped pair is
//   replaced and skipped by 2, otherwise the token is kept (:63-81); repeat until a pass makes
//   no merge (:82-85); serialise big-endian u16 (:88-91).
// out must hold 2 * n bytes.  Returns the number of output bytes.
// ---------------------------------------------------------------------------------------
size_t oracle_bpe_process_chunk(const omap *m, const uint8_t *in, size_t n, uint8_t *out) {
    if (n == 0) return 0;
    uint16_t *tok = (uint16_t *)malloc(n * sizeof(uint16_t));
    uint16_t *nxt = (uint16_t *)malloc(n * sizeof(uint16_t));
    for (size_t i = 0; i < n; ++i) tok[i] = in[i];
    size_t len = n;
    for (;;) {
        int merges_found = 0;
        size_t o = 0, i = 0;
        while (i < len) {
            uint16_t v;
            if (i < len - 1) {
                if (map_get(m, tok[i], tok[i + 1], &v)) { nxt[o++] = v; i += 2; merges_found = 1; }
                else { nxt[o++] = tok[i]; i += 1; }
            } else {
                nxt[o++] = tok[i]; i += 1;
            }
        }
        uint16_t *t = tok; tok = nxt; nxt = t;
        len = o;
        if (!merges_found) break;
    }
    for (size_t i = 0; i < len; ++i) { out[2 * i] = (uint8_t)(tok[i] >> 8); out[2 * i + 1] = (uint8_t)tok[i]; }
    free(tok);
    free(nxt);
    return 2 * len;
}

// BasicTokenizationStrategy::process_chunk — tokenizer.rs:108-124: byte b -> BE [0, b].
size_t oracle_basic_process_chunk(const uint8_t *in, size_t n, uint8_t *out) {
    for (size_t i = 0; i < n; ++i) { out[2 * i] = 0; out[2 * i + 1] = in[i]; }
    return 2 * n;
}

// PassthroughStrategy::process_chunk — tokenizer.rs:138-144: copy.
size_t oracle_passthrough_process_chunk(const uint8_t *in, size_t n, uint8_t *out) {
    memcpy(out, in, n);
    return n;
}

// ---------------------------------------------------------------------------------------
// Pipeline restatement: select_strategy (lib.rs:271-282: passthrough > BPE > basic),
// content-type token (lib.rs:93-104, :284-293), mmap chunk split (pipeline.rs:73-81),
// one task per chunk, ordered concatenation by chunk id (pipeline.rs:107-116, :153-192).
// Work is spread over `threads` pthreads (the reference uses tokio tasks; scheduling does
// not affect the bytes because results are re-ordered by chunk id).
// out capacity: 2 + 2 * n.  chunk_out_len (optional) receives each chunk's output bytes.
// ---------------------------------------------------------------------------------------
typedef struct {
    const omap *m; int passthrough;
    const uint8_t *in; size_t n; size_t cs; size_t nchunks;
    uint8_t *scratch;  // 2 * n, chunk k's result at 2 * k * cs
    size_t *lens;
    size_t next; pthread_mutex_t mu;
} run_ctx;

static void *run_worker(void *arg) {
    run_ctx *c = (run_ctx *)arg;
    for (;;) {
        pthread_mutex_lock(&c->mu);
        size_t k = c->next++;
        pthread_mutex_unlock(&c->mu);
        if (k >= c->nchunks) break;
        size_t st = k * c->cs, len = c->n - st < c->cs ? c->n - st : c->cs;
        uint8_t *dst = c->scratch + 2 * st;
        if (c->passthrough) c->lens[k] = oracle_passthrough_process_chunk(c->in + st, len, dst);
        else if (c->m) c->lens[k] = oracle_bpe_process_chunk(c->m, c->in + st, len, dst);
        else c->lens[k] = oracle_basic_process_chunk(c->in + st, len, dst);
    }
    return NULL;
}

size_t oracle_run_chunks(const omap *m, int passthrough, const uint8_t *in, size_t n, size_t chunk_size,
                         int content_token, int threads, uint8_t *out, size_t *chunk_out_len) {
    size_t o = 0;
    if (content_token >= 0) { out[0] = (uint8_t)(content_token >> 8); out[1] = (uint8_t)content_token; o = 2; }
    if (n == 0) return o;
    run_ctx c;
    memset(&c, 0, sizeof c);
    c.m = m; c.passthrough = passthrough; c.in = in; c.n = n; c.cs = chunk_size;
    c.nchunks = (n + chunk_size - 1) / chunk_size;
    c.scratch = (uint8_t *)malloc(2 * n);
    c.lens = (size_t *)calloc(c.nchunks, sizeof(size_t));
    pthread_mutex_init(&c.mu, NULL);
    if (threads < 1) threads = 1;
    if ((size_t)threads > c.nchunks) threads = (int)c.nchunks;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 1; t < threads; ++t) pthread_create(&th[t], NULL, run_worker, &c);
    run_worker(&c);
    for (int t = 1; t < threads; ++t) pthread_join(th[t], NULL);
    for (size_t k = 0; k < c.nchunks; ++k) {
        memcpy(out + o, c.scratch + 2 * k * chunk_size, c.lens[k]);
        o += c.lens[k];
        if (chunk_out_len) chunk_out_len[k] = c.lens[k];
    }
    pthread_mutex_destroy(&c.mu);
    free(th); free(c.lens); free(c.scratch);
    return o;
}

// ---------------------------------------------------------------------------------------
// "Optimised CPU" line of SURVEY.md §8(d), timed beside the faithful restatement above for
// fairness: the same greedy scan (tokenizer.rs:63-81) for a single-pass byte-pair map (no map
// value is a key component, so one pass is the fixpoint), over a dense 64K-entry table instead
// of a hash map, one pass per chunk, big-endian writes, chunks over pthreads.  Table entry
// (a << 8 | b) = value + 1, or 0 for no merge.  Baseline only: never a checker.
// ---------------------------------------------------------------------------------------
typedef struct {
    const uint32_t *tab; const uint8_t *in; size_t n; size_t cs; size_t nchunks;
    uint8_t *scratch; size_t *lens; size_t next; pthread_mutex_t mu;
} fast_ctx;

static size_t fast_chunk(const uint32_t *tab, const uint8_t *in, size_t n, uint8_t *out) {
    size_t o = 0, i = 0;
    while (i + 1 < n) {   // branch-free: the merge outcome only moves i
        const uint32_t v = tab[((uint32_t)in[i] << 8) | in[i + 1]];
        const uint32_t t = v ? v - 1 : in[i];
        out[o] = (uint8_t)(t >> 8);
        out[o + 1] = (uint8_t)t;
        o += 2;
        i += 1 + (v != 0);
    }
    if (i < n) { out[o] = 0; out[o + 1] = in[i]; o += 2; }
    return o;
}

static void *fast_worker(void *arg) {
    fast_ctx *c = (fast_ctx *)arg;
    for (;;) {
        pthread_mutex_lock(&c->mu);
        size_t k = c->next++;
        pthread_mutex_unlock(&c->mu);
        if (k >= c->nchunks) break;
        size_t st = k * c->cs, len = c->n - st < c->cs ? c->n - st : c->cs;
        c->lens[k] = fast_chunk(c->tab, c->in + st, len, c->scratch + 2 * st);
    }
    return NULL;
}

// Returns the output bytes, or (size_t)-1 when the map is not a single-pass byte-pair map.
size_t oracle_fast_run_chunks(const uint16_t *a, const uint16_t *b, const uint16_t *v, size_t nm, const uint8_t *in,
                              size_t n, size_t chunk_size, int threads, uint8_t *out) {
    uint32_t *tab = (uint32_t *)calloc(65536, sizeof(uint32_t));
    uint8_t *comp = (uint8_t *)calloc(65536, 1);
    for (size_t i = 0; i < nm; ++i) {
        if (a[i] > 255 || b[i] > 255) { free(tab); free(comp); return (size_t)-1; }
        tab[((uint32_t)a[i] << 8) | b[i]] = (uint32_t)v[i] + 1;   // a later duplicate overwrites
        comp[a[i]] = comp[b[i]] = 1;
    }
    for (size_t i = 0; i < nm; ++i)
        if (comp[v[i]]) { free(tab); free(comp); return (size_t)-1; }
    free(comp);
    if (n == 0) { free(tab); return 0; }
    fast_ctx c;
    memset(&c, 0, sizeof c);
    c.tab = tab; c.in = in; c.n = n; c.cs = chunk_size;
    c.nchunks = (n + chunk_size - 1) / chunk_size;
    c.scratch = (uint8_t *)malloc(2 * n);
    c.lens = (size_t *)calloc(c.nchunks, sizeof(size_t));
    pthread_mutex_init(&c.mu, NULL);
    if (threads < 1) threads = 1;
    if ((size_t)threads > c.nchunks) threads = (int)c.nchunks;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 1; t < threads; ++t) pthread_create(&th[t], NULL, fast_worker, &c);
    fast_worker(&c);
    for (int t = 1; t < threads; ++t) pthread_join(th[t], NULL);
    size_t o = 0;
    for (size_t k = 0; k < c.nchunks; ++k) { memcpy(out + o, c.scratch + 2 * k * chunk_size, c.lens[k]); o += c.lens[k]; }
    pthread_mutex_destroy(&c.mu);
    free(th); free(c.lens); free(c.scratch); free(tab);
    return o;
}

// ---------------------------------------------------------------------------------------
// parse_chunk_size_str — blt_core/src/utils.rs:10-45.  KB/MB are 1024-based, raw digits are
// bytes; the multiply wraps (release build).  Returns 0 ok, 1 error (msg = reference text).
// ---------------------------------------------------------------------------------------
static size_t trim_front(const unsigned char *s, size_t n) {
    size_t i = 0; uint32_t cp;
    while (i < n) { int l = utf8_decode(s + i, n - i, &cp); if (!l || !uni_space(cp)) break; i += (size_t)l; }
    return i;
}

static size_t trim_back(const unsigned char *s, size_t n) {  // returns new length
    while (n > 0) {
        size_t j = n - 1;
        while (j > 0 && (s[j] & 0xC0) == 0x80) --j;
        uint32_t cp;
        int l = utf8_decode(s + j, n - j, &cp);
        if (!l || (size_t)l != n - j || !uni_space(cp)) break;
        n = j;
    }
    return n;
}

// <usize as FromStr>: optional '+', ASCII digits, checked overflow.
static int parse_usize(const unsigned char *s, size_t n, uint64_t *out) {
    if (n == 0) return 3;
    size_t i = 0;
    if (s[0] == '+' || s[0] == '-') { if (n == 1) return 1; if (s[0] == '+') i = 1; }
    uint64_t r = 0;
    for (; i < n; ++i) {
        int mul_ok = r <= UINT64_MAX / 10;
        if (s[i] < '0' || s[i] > '9') return 1;
        if (!mul_ok) return 2;
        r *= 10;
        uint64_t d = (uint64_t)(s[i] - '0');
        if (r > UINT64_MAX - d) return 2;
        r += d;
    }
    *out = r;
    return 0;
}

int oracle_parse_chunk_size(const char *str, uint64_t *out, char *msg, size_t msgcap) {
    const unsigned char *s = (const unsigned char *)str;
    size_t n = strlen(str);
    size_t f = trim_front(s, n);
    s += f; n -= f;
    n = trim_back(s, n);
    char *t = (char *)malloc(n + 1);
    memcpy(t, s, n); t[n] = 0;
    int rc = 0;
    if (n == 0) { set_msg(msg, msgcap, "Input string is empty%s%s", "", ""); free(t); return 1; }
    int has_unit = 0, all_digits = 1;
    if (n >= 2) {
        char u0 = t[n - 2], u1 = t[n - 1];
        if ((u0 == 'k' || u0 == 'K' || u0 == 'm' || u0 == 'M') && (u1 == 'b' || u1 == 'B')) has_unit = 1;
    }
    for (size_t i = 0; i < n; ++i) if (t[i] < '0' || t[i] > '9') { all_digits = 0; break; }
    size_t numlen;
    uint64_t mult;
    if (has_unit) {
        numlen = n - 2;
        mult = (t[n - 2] == 'k' || t[n - 2] == 'K') ? 1024ULL : 1024ULL * 1024ULL;
        if (numlen == 0) {
            char unit[3] = {t[n - 2], t[n - 1], 0};
            set_msg(msg, msgcap, "Number part missing for unit '%s'%s", unit, "");
            free(t); return 1;
        }
    } else if (all_digits) {
        numlen = n; mult = 1;
    } else {
        set_msg(msg, msgcap,
                "Invalid unit or format: '%s'. Number must be followed by KB, MB, or be raw bytes.%s", t, "");
        free(t); return 1;
    }
    uint64_t num;
    if (parse_usize((const unsigned char *)t, numlen, &num) != 0) {
        char *np = (char *)malloc(numlen + 1);
        memcpy(np, t, numlen); np[numlen] = 0;
        set_msg(msg, msgcap, "Invalid number: '%s'%s", np, "");
        free(np); free(t); return 1;
    }
    *out = num * mult;  // wrapping multiply (release)
    free(t);
    return rc;
}

// get_effective_chunk_size — blt_core/src/chunking.rs:26-62.
// has_cli: --chunksize given.  total_ram: sysinfo total_memory() in bytes (dynamic branch
// only; parity unpinned there, the reference bounds-tests it only).
uint64_t oracle_effective_chunk_size(int has_cli, uint64_t cli, uint64_t threads, unsigned memcap,
                                     uint64_t total_ram) {
    const uint64_t amin = 256 * 1024, amax = 128ULL * 1024 * 1024;
    const uint64_t dmin = 1024 * 1024, dmax = 16ULL * 1024 * 1024;
    if (has_cli) return cli < amin ? amin : (cli > amax ? amax : cli);
    uint64_t usable = (uint64_t)((double)total_ram * ((double)memcap / 100.0));
    uint64_t per_thread = usable / (threads ? threads : 1);
    uint64_t c = per_thread / 4;
    c = c < dmin ? dmin : (c > dmax ? dmax : c);
    c = c < amin ? amin : (c > amax ? amax : c);
    return c;
}

// determine_thread_count — blt_core/src/utils.rs:79-97.  has_cli=0 -> logical CPUs.
uint64_t oracle_thread_count(int has_cli, uint64_t threads) {
    if (has_cli) return threads == 0 ? 1 : threads;
    long c = sysconf(_SC_NPROCESSORS_ONLN);
    return c > 0 ? (uint64_t)c : 1;
}
