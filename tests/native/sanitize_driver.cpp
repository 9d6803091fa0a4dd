// Host-sanitizer driver of the C ABI (an ASan/UBSan build of the host library).
// Test infrastructure: built by `make sanitize` with the host code of libblt_bpe instrumented
// (-Xarch_host -fsanitize=address,undefined; device code is not instrumented) and linked with the
// C oracle (oracle/bpe_oracle.c, the checker).  Every check compares the library with the oracle.
//
//   build/san/blt_sanitize_driver [--cpu]    exit 0 = every check passed and no sanitizer report
//
// --cpu (or no HIP device): the host-only entry points — chunk-size parsing and clamping, thread
// count, the merges loader on valid, invalid, wrapping, missing and directory paths, handle
// creation, info and workspace sizes, null-argument errors.  With a device, also process_chunk /
// process_chunks / basic / run_tokenizer against the oracle, and 8 threads sharing one handle.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/blt_bpe.h"

extern "C" {
struct omap;
int oracle_load_merges(const char* path, uint16_t* ka, uint16_t* kb, uint16_t* kv, size_t cap, size_t* n_out,
                       char* msg, size_t msgcap);
omap* oracle_map_new(const uint16_t* a, const uint16_t* b, const uint16_t* v, size_t n);
void oracle_map_free(omap* m);
size_t oracle_bpe_process_chunk(const omap* m, const uint8_t* in, size_t n, uint8_t* out);
size_t oracle_basic_process_chunk(const uint8_t* in, size_t n, uint8_t* out);
size_t oracle_run_chunks(const omap* m, int passthrough, const uint8_t* in, size_t n, size_t chunk_size,
                         int content_token, int threads, uint8_t* out, size_t* chunk_out_len);
int oracle_parse_chunk_size(const char* str, uint64_t* out, char* msg, size_t msgcap);
uint64_t oracle_effective_chunk_size(int has_cli, uint64_t cli, uint64_t threads, unsigned memcap, uint64_t ram);
uint64_t oracle_thread_count(int has_cli, uint64_t threads);
}

static int g_fail = 0;
#define CHECK(cond, ...)                                      \
    do {                                                      \
        if (!(cond)) {                                        \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                     \
            fprintf(stderr, "\n");                            \
            ++g_fail;                                         \
        }                                                     \
    } while (0)

static std::string tmpdir;

static std::string write_file(const char* name, const std::string& body) {
    std::string p = tmpdir + "/" + name;
    FILE* f = fopen(p.c_str(), "wb");
    fwrite(body.data(), 1, body.size(), f);
    fclose(f);
    return p;
}

static void check_parse() {
    const char* cases[] = {"16MB", "256KB", "1KB", "1MB", "0", "", "abc", "1.5MB", "10GB", " 1MB", "1mb", "12",
                           "18446744073709551615", "18446744073709551616", "99999999999999999MB", "MB", "KB1"};
    for (const char* c : cases) {
        uint64_t a = 0, b = 0;
        char msg[256];
        const int ra = blt_parse_chunk_size(c, &a);
        const int rb = oracle_parse_chunk_size(c, &b, msg, sizeof msg);
        CHECK((ra == 0) == (rb == 0), "parse '%s': rc %d vs oracle %d", c, ra, rb);
        if (ra == 0 && rb == 0) CHECK(a == b, "parse '%s': %llu vs %llu", c, (unsigned long long)a, (unsigned long long)b);
        if (ra != 0) CHECK(blt_last_error() && *blt_last_error(), "parse '%s': empty error text", c);
    }
    for (uint64_t cli : {0ull, 1ull, 262143ull, 262144ull, 1ull << 20, 1ull << 27, (1ull << 27) + 1, ~0ull})
        CHECK(blt_effective_chunk_size(1, cli, 8, 80) == oracle_effective_chunk_size(1, cli, 8, 80, 0),
              "effective chunk size (cli %llu)", (unsigned long long)cli);
    for (uint64_t t : {0ull, 1ull, 7ull, 1000ull})
        CHECK(blt_determine_thread_count(1, t) == oracle_thread_count(1, t), "thread count %llu", (unsigned long long)t);
    CHECK(blt_determine_thread_count(0, 0) >= 1, "auto thread count");
}

static void check_loader() {
    std::string wrap;
    for (int i = 0; i < 65536; ++i) wrap += std::to_string((i >> 8) & 255) + " " + std::to_string(i & 255) + "\n";
    wrap += "1 2\n";
    struct Case { const char* name; std::string body; };
    const Case cases[] = {
        {"ok.txt", "97 98\n98 99\n\n# comment\n97 98\n"},
        {"crlf.txt", "1 2\r\n3 4\r\n"},
        {"bad_fields.txt", "1 2 3\n"},
        {"bad_value.txt", "300 1\n"},
        {"bad_neg.txt", "-1 2\n"},
        {"one_field.txt", "7\n"},
        {"empty.txt", ""},
        {"utf8.txt", "1 2\n\xff\xfe\n"},
        {"wrap.txt", wrap},
    };
    std::vector<uint16_t> a(70000), b(70000), v(70000), oa(70000), ob(70000), ov(70000);
    for (const Case& c : cases) {
        const std::string p = write_file(c.name, c.body);
        size_t n = 0, on = 0;
        char msg[512];
        const int ra = blt_load_bpe_merges(p.c_str(), a.data(), b.data(), v.data(), a.size(), &n);
        const int rb = oracle_load_merges(p.c_str(), oa.data(), ob.data(), ov.data(), oa.size(), &on, msg, sizeof msg);
        CHECK((ra == 0) == (rb == 0), "loader %s: rc %d vs oracle %d", c.name, ra, rb);
        if (ra == 0 && rb == 0) {
            CHECK(n == on, "loader %s: %zu vs %zu entries", c.name, n, on);
            for (size_t i = 0; i < n && i < on; ++i)
                CHECK(a[i] == oa[i] && b[i] == ob[i] && v[i] == ov[i], "loader %s: entry %zu", c.name, i);
            blt_bpe* h = nullptr;
            CHECK(blt_bpe_create_from_file(p.c_str(), &h) == 0 && h, "create_from_file %s", c.name);
            size_t ne = 0;
            int sp = -1;
            CHECK(h && blt_bpe_info(h, &ne, &sp) == 0 && ne == n, "info %s", c.name);
            if (h) {
                for (uint64_t sz : {1ull, 4096ull, 1ull << 20, 5ull << 30})
                    CHECK(blt_bpe_workspace_size(h, sz, 1 << 20) > 0, "workspace size %llu", (unsigned long long)sz);
                blt_bpe_destroy(h);
            }
        } else {
            CHECK(blt_last_error() && *blt_last_error(), "loader %s: empty error text", c.name);
        }
    }
    size_t n = 0;
    const std::string missing = tmpdir + "/missing.txt";
    CHECK(blt_load_bpe_merges(missing.c_str(), a.data(), b.data(), v.data(), a.size(), &n) == BLT_E_NOT_FOUND,
          "missing file");
    CHECK(blt_load_bpe_merges(tmpdir.c_str(), a.data(), b.data(), v.data(), a.size(), &n) != 0, "directory path");
    CHECK(strstr(blt_last_error(), "os error") != nullptr, "directory error text: %s", blt_last_error());
    blt_bpe* h = nullptr;
    CHECK(blt_bpe_create_from_file(tmpdir.c_str(), &h) != 0 && !h, "create_from_file on a directory");
    const std::string ok = tmpdir + "/ok.txt";
    CHECK(blt_load_bpe_merges(ok.c_str(), a.data(), b.data(), v.data(), 1, &n) == BLT_E_NOSPC && n == 2, "cap too small");
}

static void check_args() {
    blt_bpe* h = nullptr;
    uint16_t a = 1, b = 2, v = 300;
    CHECK(blt_bpe_create(&a, &b, &v, 1, 1u, &h) != 0, "nonzero flags");
    CHECK(blt_bpe_create(&a, &b, &v, 1, 0, nullptr) != 0, "null out");
    CHECK(blt_parse_chunk_size(nullptr, nullptr) != 0, "null parse");
    CHECK(blt_bpe_info(nullptr, nullptr, nullptr) != 0, "null info");
    CHECK(blt_run_tokenizer(nullptr) != 0, "null run config");
    blt_bpe_destroy(nullptr);
}

static std::vector<uint8_t> oracle_chunk(const omap* m, const std::vector<uint8_t>& in) {
    std::vector<uint8_t> out(2 * in.size() + 2);
    out.resize(oracle_bpe_process_chunk(m, in.data(), in.size(), out.data()));
    return out;
}

static void check_device() {
    std::mt19937_64 rng(7);
    for (int trial = 0; trial < 6; ++trial) {
        // maps over a small alphabet: single-pass files, chained and byte-valued (general) maps
        const int alph = 4 + trial * 3;
        std::vector<uint16_t> a, b, v;
        for (int i = 0; i < 40; ++i) {
            a.push_back(rng() % alph);
            b.push_back(trial & 1 ? 256 + rng() % 8 : rng() % alph);
            v.push_back(trial % 3 == 2 ? rng() % alph : 256 + rng() % 64);
        }
        blt_bpe* h = nullptr;
        CHECK(blt_bpe_create(a.data(), b.data(), v.data(), a.size(), 0, &h) == 0, "create trial %d", trial);
        omap* m = oracle_map_new(a.data(), b.data(), v.data(), a.size());
        for (size_t n : {0ul, 1ul, 17ul, 4095ul, 70001ul, 1ul << 20}) {
            std::vector<uint8_t> in(n);
            for (auto& c : in) c = rng() % alph;
            std::vector<uint8_t> out(2 * n + 2);
            size_t len = 0;
            const int prc = blt_bpe_process_chunk(h, in.data(), n, out.data(), out.size(), &len);
            CHECK(prc == 0, "process_chunk %zu: rc %d, %s", n, prc, prc ? blt_last_error() : "");
            out.resize(len);
            CHECK(out == oracle_chunk(m, in), "process_chunk %zu bytes, trial %d", n, trial);
            for (size_t cs : {4096ul, 65537ul}) {
                std::vector<uint8_t> got(2 * n + 2), exp(2 * n + 2);
                std::vector<uint64_t> lens((n + cs - 1) / cs + 1);
                std::vector<size_t> elens(lens.size());
                size_t gl = 0;
                const int crc = blt_bpe_process_chunks(h, in.data(), n, cs, 2, got.data(), got.size(), &gl, lens.data());
                CHECK(crc == 0, "process_chunks %zu cs %zu: rc %d, %s", n, cs, crc, crc ? blt_last_error() : "");
                const size_t el = oracle_run_chunks(m, 0, in.data(), n, cs, -1, 2, exp.data(), elens.data());
                CHECK(gl == el && memcmp(got.data(), exp.data(), gl) == 0, "process_chunks %zu cs %zu", n, cs);
            }
        }
        // 8 threads share the handle (the reference's Arc<dyn TokenizationStrategy>)
        std::vector<std::thread> th;
        std::vector<int> ok(8, 0);
        for (int t = 0; t < 8; ++t)
            th.emplace_back([&, t] {
                std::mt19937_64 r(100 + t);
                std::vector<uint8_t> in(30000 + 1000 * t);
                for (auto& c : in) c = r() % alph;
                std::vector<uint8_t> out(2 * in.size());
                size_t len = 0;
                ok[t] = blt_bpe_process_chunk(h, in.data(), in.size(), out.data(), out.size(), &len) == 0 &&
                        std::vector<uint8_t>(out.begin(), out.begin() + len) == oracle_chunk(m, in);
            });
        for (auto& x : th) x.join();
        for (int t = 0; t < 8; ++t) CHECK(ok[t], "thread %d", t);
        // run_tokenizer: file in, file out, the content-type token first
        std::vector<uint8_t> in(300000);
        for (auto& c : in) c = rng() % alph;
        const std::string ip = write_file("run_in.bin", std::string(in.begin(), in.end()));
        const std::string op = tmpdir + "/run_out.bin";
        blt_run_config cfg;
        memset(&cfg, 0, sizeof cfg);
        cfg.input_path = ip.c_str();
        cfg.output_path = op.c_str();
        cfg.bpe = h;
        cfg.content_token = BLT_CONTENT_TEXT;
        cfg.threads = 4;
        cfg.chunk_size = 65536;
        CHECK(blt_run_tokenizer(&cfg) == 0, "run_tokenizer: %s", blt_last_error());
        std::vector<uint8_t> exp(2 * in.size() + 2);
        exp.resize(oracle_run_chunks(m, 0, in.data(), in.size(), 65536, BLT_CONTENT_TEXT, 4, exp.data(), nullptr));
        FILE* f = fopen(op.c_str(), "rb");
        std::vector<uint8_t> got(exp.size() + 16);
        got.resize(f ? fread(got.data(), 1, got.size(), f) : 0);
        if (f) fclose(f);
        CHECK(got == exp, "run_tokenizer output (%zu vs %zu bytes)", got.size(), exp.size());
        oracle_map_free(m);
        blt_bpe_destroy(h);
    }
    std::vector<uint8_t> in(100001), out(2 * in.size()), exp(2 * in.size());
    for (size_t i = 0; i < in.size(); ++i) in[i] = (uint8_t)(i * 131);
    size_t len = 0;
    CHECK(blt_basic_process_chunk(in.data(), in.size(), out.data(), out.size(), &len) == 0, "basic");
    CHECK(len == oracle_basic_process_chunk(in.data(), in.size(), exp.data()) && out == exp, "basic output");
}

int main(int argc, char** argv) {
    bool cpu = argc > 1 && strcmp(argv[1], "--cpu") == 0;
    char tmpl[] = "/tmp/blt_san_XXXXXX";
    if (!mkdtemp(tmpl)) return 2;
    tmpdir = tmpl;
    CHECK(blt_version() && *blt_version(), "version");
    check_parse();
    check_loader();
    check_args();
    if (!cpu) {
        uint16_t a = 1, b = 2, v = 300;
        blt_bpe* h = nullptr;
        uint8_t in[2] = {1, 2}, out[4];
        size_t len = 0;
        blt_bpe_create(&a, &b, &v, 1, 0, &h);
        const int rc = blt_bpe_process_chunk(h, in, 2, out, 4, &len);
        blt_bpe_destroy(h);
        if (rc == BLT_E_NODEV) {
            // no device, or a HIP runtime that did not come up in this process (under ASan the
            // runtime's start-up fails now and then, as ASan's shadow mappings land where it
            // needs address space): host-only checks, and the message says why
            printf("no HIP device: host-only checks (probe rc %d: %s)\n", rc, blt_last_error());
            cpu = true;
        } else if (rc != 0) {
            // a device that is there but failed the probe (a kernel fault, a sticky error, a broken
            // launch) is a failure, not a reason to skip the device checks
            CHECK(false, "device probe: rc %d, %s", rc, blt_last_error());
            cpu = true;
        } else {
            check_device();
        }
    }
    std::string rm = "rm -rf " + tmpdir;
    if (system(rm.c_str())) {}
    printf("%s: %d failure(s)\n", cpu ? "host checks" : "host and device checks", g_fail);
    fflush(stdout);
    // exit without the HIP runtime's static teardown (as the blt CLI does): ASan flags a
    // mismatched delete inside libhsa-runtime64's own finalizers, which is not this library's code
    _exit(g_fail ? 1 : 0);
}
