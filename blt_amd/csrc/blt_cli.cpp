// blt — command-line drop-in for jtrefon/blt's `blt` binary (src/main.rs:8-60), over the C ABI
// of libblt_bpe.so (include/blt_bpe.h).  Same flags, same defaults, same output bytes:
//
//   -i/--input FILE        input file (mmap); absent: stdin       (main.rs:11-17, io_handler.rs:55-62)
//   -o/--output FILE       output file; absent: stdout            (main.rs:19-25, io_handler.rs:70-78)
//   --merges FILE          BPE merges file -> BpeStrategy        (main.rs:27-32, lib.rs:271-282)
//   --passthrough          copy input unchanged                  (main.rs:34-35, tokenizer.rs:129-137)
//   --type text|audio|bin|video   prepend 0xFF01..0xFF04 (BE)   (main.rs:37-38, lib.rs:96-107, :284-293)
//   --threads N            chunks in flight (0 -> 1; default: num_cpus)   (utils.rs:83-101)
//   --memcap PERCENT       RAM share for the automatic chunk size (default 80)  (lib.rs:172)
//   --chunksize SIZE       "4MB", "256KB", raw bytes; clamped to [256 KiB, 128 MiB] (chunking.rs:26-31)
// plus one MI355X option:
//   --gpus N               devices the file path shards its chunks over (default: all visible)
// "-" is a file name, as in the reference (clap passes it through and File::open opens a file
// named "-"); the standard streams are used when -i / -o are absent.
//
// CoreConfig::new_from_cli (lib.rs:149-174) is resolved here (thread count, chunk size, merges
// file); run_tokenizer (lib.rs:246-267) and its pipeline run in the library (blt_run_tokenizer,
// blt_pipeline.cpp).  Tokenising runs on the GPU only (there is no CPU fallback).
// Errors: configuration errors print "Error: <message>" and exit 1 (main's io::Result); pipeline
// errors print "Error running tokenizer: <message>" and exit 1 (main.rs:99-102).
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <string>

#include "../../include/blt_bpe.h"

namespace {

struct Args {
    std::string input, output, merges;
    bool has_input = false, has_output = false, has_merges = false, passthrough = false;
    int content_token = -1;
    bool has_threads = false;
    uint64_t threads = 0;
    uint32_t memcap = 80;
    bool has_chunksize = false;
    std::string chunksize;
    int gpus = 0;   // 0: all visible
};

[[noreturn]] void usage(FILE* f, int code) {
    fprintf(f,
            "Usage: blt [OPTIONS]\n\n"
            "Options:\n"
            "  -i, --input <FILE>         Input file path (stdin if absent)\n"
            "  -o, --output <FILE>        Output file path (stdout if absent)\n"
            "      --merges <FILE>        BPE merges file for advanced tokenization\n"
            "      --passthrough          Use passthrough mode (copy file without tokenization)\n"
            "      --type <TYPE>          Prepend content-type token [possible values: text, audio, bin, video]\n"
            "      --threads <NUM>        Override worker count (default: auto based on cores)\n"
            "      --memcap <PERCENT>     Max RAM usage fraction (e.g., 70 for 70%%)\n"
            "      --chunksize <SIZE>     Min/Max chunk size (e.g. 4MB, 256KB).\n"
            "      --gpus <NUM>           GPUs the file path shards its chunks over (default: all)\n"
            "  -h, --help                 Print help\n"
            "  -V, --version              Print version\n");
    exit(code);
}

[[noreturn]] void arg_error(const char* fmt, const char* a) {
    fprintf(stderr, "error: ");
    fprintf(stderr, fmt, a);
    fprintf(stderr, "\n\nFor more information, try '--help'.\n");
    exit(2);   // clap's usage-error exit code
}

bool parse_u64(const char* s, uint64_t* v) {
    if (!*s) return false;
    char* end = nullptr;
    errno = 0;
    unsigned long long x = strtoull(s, &end, 10);
    if (errno || *end || s[0] == '-' || s[0] == '+') return false;
    *v = x;
    return true;
}

Args parse_args(int argc, char** argv) {
    Args a;
    for (int i = 1; i < argc; ++i) {
        std::string k = argv[i], val;
        bool has_val = false;
        const size_t eq = k.find('=');
        if (k.rfind("--", 0) == 0 && eq != std::string::npos) {
            val = k.substr(eq + 1);
            k = k.substr(0, eq);
            has_val = true;
        }
        auto take = [&](const char* name) -> std::string {
            if (has_val) return val;
            if (i + 1 >= argc) arg_error("a value is required for '%s' but none was supplied", name);
            return argv[++i];
        };
        if (k == "-h" || k == "--help") usage(stdout, 0);
        if (k == "-V" || k == "--version") {
            printf("%s\n", blt_version());
            exit(0);
        }
        if (k == "-i" || k == "--input") {
            a.input = take("--input <FILE>");
            a.has_input = true;
        } else if (k == "-o" || k == "--output") {
            a.output = take("--output <FILE>");
            a.has_output = true;
        } else if (k == "--merges") {
            a.merges = take("--merges <FILE>");
            a.has_merges = true;
        } else if (k == "--passthrough") {
            a.passthrough = true;
        } else if (k == "--type") {
            const std::string t = take("--type <TYPE>");
            static const char* names[] = {"text", "audio", "bin", "video"};
            a.content_token = -1;
            for (int j = 0; j < 4; ++j)
                if (t == names[j]) a.content_token = 0xFF01 + j;   // lib.rs:96-107
            if (a.content_token < 0) arg_error("invalid value '%s' for '--type <TYPE>'", t.c_str());
        } else if (k == "--threads") {
            const std::string t = take("--threads <NUM>");
            if (!parse_u64(t.c_str(), &a.threads)) arg_error("invalid value '%s' for '--threads <NUM>'", t.c_str());
            a.has_threads = true;
        } else if (k == "--memcap") {
            const std::string t = take("--memcap <PERCENT>");
            uint64_t m = 0;
            if (!parse_u64(t.c_str(), &m) || m > 255) arg_error("invalid value '%s' for '--memcap <PERCENT>'", t.c_str());
            a.memcap = (uint32_t)m;   // u8 in the reference
        } else if (k == "--chunksize") {
            a.chunksize = take("--chunksize <SIZE>");
            a.has_chunksize = true;
        } else if (k == "--gpus") {
            const std::string t = take("--gpus <NUM>");
            uint64_t g = 0;
            if (!parse_u64(t.c_str(), &g) || g > 64) arg_error("invalid value '%s' for '--gpus <NUM>'", t.c_str());
            a.gpus = (int)g;
        } else {
            arg_error("unexpected argument '%s' found", argv[i]);
        }
    }
    return a;
}

[[noreturn]] void config_error(const std::string& msg) {
    fprintf(stderr, "Error: %s\n", msg.c_str());
    exit(1);
}

[[noreturn]] void run_error(const std::string& msg) {
    fprintf(stderr, "Error running tokenizer: %s\n", msg.c_str());
    exit(1);
}

std::string lib_error(int rc) {
    const char* m = blt_last_error();
    return (m && *m) ? std::string(m) : ("error " + std::to_string(rc));
}

}  // namespace

static double mono_now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Seconds from the process's start (exec) to now: /proc/self/stat's starttime (clock ticks since
// boot) against CLOCK_BOOTTIME.  BLT_CLI_TIMING only: the exec, dynamic loading (the HIP runtime
// libraries) and static constructors before main.
static double since_exec() {
    FILE* f = fopen("/proc/self/stat", "r");
    if (!f) return -1.0;
    char buf[2048];
    const size_t len = fread(buf, 1, sizeof buf - 1, f);
    fclose(f);
    buf[len] = 0;
    const char* q = strrchr(buf, ')');   // comm may hold spaces
    if (!q) return -1.0;
    unsigned long long start = 0;
    int field = 2;
    for (const char* c = q + 1; *c; ++c) {
        if (*c == ' ') {
            ++field;
            if (field == 22) { start = strtoull(c + 1, nullptr, 10); break; }
        }
    }
    timespec bt;
    clock_gettime(CLOCK_BOOTTIME, &bt);
    return (double)bt.tv_sec + 1e-9 * (double)bt.tv_nsec - (double)start / (double)sysconf(_SC_CLK_TCK);
}

int main(int argc, char** argv) {
    blt_log_init_from_env();   // tracing_subscriber::fmt().with_env_filter(RUST_LOG) (main.rs:83-85)
    const double t_main = mono_now();
    const double t_exec = getenv("BLT_CLI_TIMING") ? since_exec() : 0.0;
    const Args a = parse_args(argc, argv);

    // CoreConfig::new_from_cli (lib.rs:149-174): threads, chunk size string, merges file
    const uint64_t threads = blt_determine_thread_count(a.has_threads ? 1 : 0, a.threads);
    uint64_t cli_cs = 0;
    if (a.has_chunksize) {
        const int rc = blt_parse_chunk_size(a.chunksize.c_str(), &cli_cs);
        if (rc) config_error(lib_error(rc));
    }
    blt_bpe* h = nullptr;
    if (a.has_merges) {
        // loaded (and validated) even when --passthrough wins the strategy choice (lib.rs:184-201)
        const int rc = blt_bpe_create_from_file(a.merges.c_str(), &h);
        if (rc) config_error(lib_error(rc));   // "Failed to load BPE merges: ..." (lib.rs:195-201)
    }
    const uint64_t cs = blt_effective_chunk_size(a.has_chunksize ? 1 : 0, cli_cs, threads, a.memcap);

    blt_run_config cfg = {};
    cfg.input_path = a.has_input ? a.input.c_str() : nullptr;
    cfg.output_path = a.has_output ? a.output.c_str() : nullptr;
    cfg.bpe = a.passthrough ? nullptr : h;
    cfg.passthrough = a.passthrough ? 1 : 0;
    cfg.content_token = a.content_token >= 0 ? (uint32_t)a.content_token : 0u;
    cfg.threads = threads;
    cfg.chunk_size = cs;
    cfg.n_gpus = a.gpus;
    const double t_run = mono_now();
    if (getenv("BLT_CLI_TIMING"))
        fprintf(stderr, "blt timing: exec -> main %.4f s, merges loaded at %.4f s\n", t_exec, t_run - t_main);
    const int rc = blt_run_tokenizer(&cfg);
    const double t_done = mono_now();
    if (rc) run_error(lib_error(rc));
    // (the handle's host and device memory go with the process: _exit below)
    if (getenv("BLT_CLI_TIMING"))
        fprintf(stderr, "blt timing: main at %.4f (monotonic), setup %.4f s, run %.4f s, teardown from %.4f\n", t_main,
                t_run - t_main, t_done - t_run, t_done);
    // Every byte is written and the output closed: leave without the HIP runtime's exit-time
    // teardown of the device contexts and pinned buffers (~0.4 s).
    fflush(nullptr);
    _exit(0);
}
