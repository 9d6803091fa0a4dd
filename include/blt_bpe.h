/*
 * blt_bpe.h — C ABI of the MI355X-native BPE merge scan (drop-in for jtrefon/blt's BPE path).
 *
 * The reference's boundary for this path is the Rust strategy trait
 *     #[async_trait] pub trait TokenizationStrategy: Send + Sync {
 *         async fn process_chunk(&self, chunk_data: &[u8]) -> io::Result<Vec<u8>>;
 *     }                                                  (blt_core/src/tokenizer.rs:21-31)
 * with BpeStrategy::new(Arc<BpeMerges>) (tokenizer.rs:43-51), BpeMerges =
 * HashMap<(u16, u16), u16> (lib.rs:75), the merges loader (config_loader.rs:14-46), and the
 * chunked pipeline that calls process_chunk once per fixed-size chunk and concatenates results
 * in chunk order (pipeline.rs:73-81, :141-168).  Every entry point below names the reference
 * item it replaces.  Plain pointers and sizes only; no C++ or torch types cross the boundary.
 *
 * Return convention: 0 on success, a negative errno on failure, with a message for the calling
 * thread in blt_last_error().  A failing HIP call is -EIO.  The library has no CPU fallback:
 * every tokenising entry point runs on the GPU and fails with -ENODEV when none is present.
 *
 * Threading: a blt_bpe handle is immutable after creation (device copies of its tables are
 * made once per device, internally synchronised), so all calls are reentrant and may run
 * concurrently from many threads, as the reference's tokio tasks call one Arc'd strategy.
 */
#ifndef BLT_BPE_H
#define BLT_BPE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BLT_ABI_VERSION 1

/* Error kinds of the reference's io::Error, as negative errno values. */
#define BLT_E_NOT_FOUND (-2)      /* -ENOENT:  io::ErrorKind::NotFound                       */
#define BLT_E_INVALID_DATA (-74)  /* -EBADMSG: io::ErrorKind::InvalidData (merges file)      */
#define BLT_E_INVALID_INPUT (-22) /* -EINVAL:  io::ErrorKind::InvalidInput / bad argument     */
#define BLT_E_NOSPC (-28)         /* -ENOSPC:  caller's output buffer too small               */
#define BLT_E_NOMEM (-12)         /* -ENOMEM                                                 */
#define BLT_E_IO (-5)             /* -EIO:     HIP runtime failure / other io::Error          */
#define BLT_E_NODEV (-19)         /* -ENODEV:  no GPU                                        */

/* Content-type tokens written big-endian before the first chunk (lib.rs:93-104, :284-293). */
#define BLT_CONTENT_TEXT 0xFF01u
#define BLT_CONTENT_AUDIO 0xFF02u
#define BLT_CONTENT_BIN 0xFF03u
#define BLT_CONTENT_VIDEO 0xFF04u

typedef struct blt_bpe blt_bpe;

/* Library version string ("blt-mi355x <semver>"; the reference reports its crate version via
 * blt_python's version(), blt_python/src/lib.rs:212-215). */
const char *blt_version(void);

/* Message of the last failing call on this thread ("" if none). */
const char *blt_last_error(void);

/* ---------------------------------------------------------------------------------------
 * Configuration helpers (CPU; they only parse and compute sizes).
 * ------------------------------------------------------------------------------------- */

/* load_bpe_merges_from_path (config_loader.rs:14-46): reads a merges file into the map's
 * entries, sorted by (a, b).  Line i (valid, 0-based) maps (u8, u8) to 256 + i with a wrapping
 * u16 counter; duplicates overwrite; empty and '#'-first lines are skipped; anything but two
 * whitespace-separated u8 values is BLT_E_INVALID_DATA with the reference's message.  A missing
 * file is BLT_E_NOT_FOUND.  If cap is too small: BLT_E_NOSPC with *n_out = entries needed. */
int blt_load_bpe_merges(const char *path, uint16_t *a, uint16_t *b, uint16_t *v, size_t cap, size_t *n_out);

/* parse_chunk_size_str (utils.rs:10-45): "16MB", "256KB", raw digits; KB/MB are 1024-based. */
int blt_parse_chunk_size(const char *s, uint64_t *out);

/* get_effective_chunk_size (chunking.rs:26-62): has_cli -> clamp(cli, 256 KiB, 128 MiB);
 * otherwise clamp(RAM * memcap% / threads / 4, 1 MiB, 16 MiB) from /proc/meminfo MemTotal. */
uint64_t blt_effective_chunk_size(int has_cli, uint64_t cli_chunk_size, uint64_t threads, uint32_t memcap_percent);

/* determine_thread_count (utils.rs:79-97): has_cli -> max(threads, 1); else num_cpus::get()
 * (num_cpus 1.17): the cgroup CPU quota (ceil(quota / period)) if one is set, otherwise the CPUs
 * in this process's affinity mask. */
uint64_t blt_determine_thread_count(int has_cli, uint64_t threads);

/* ---------------------------------------------------------------------------------------
 * Strategy handle: BpeStrategy::new(Arc<BpeMerges>) (tokenizer.rs:43-51).
 * ------------------------------------------------------------------------------------- */

/* Builds the strategy from n map entries (a[i], b[i]) -> v[i]; a later duplicate key
 * overwrites an earlier one (HashMap collect).  flags must be 0. */
int blt_bpe_create(const uint16_t *a, const uint16_t *b, const uint16_t *v, size_t n, uint32_t flags,
                   blt_bpe **out);

/* CoreConfig::load_bpe_data + BpeStrategy::new (lib.rs:184-201, :271-282): loads a merges file
 * with exactly the semantics of blt_load_bpe_merges and builds the strategy. */
int blt_bpe_create_from_file(const char *merges_path, blt_bpe **out);

void blt_bpe_destroy(blt_bpe *h);

/* Device errors are sticky per handle: when a kernel of h flags an error (look-back timeout,
 * output range or prefix invariant; its output is then invalid), every later call taking h fails
 * with BLT_E_IO until this call, which returns BLT_E_IO once if such an error was recorded (and
 * clears it), 0 otherwise.  The reference's strategy never fails mid-run; a failed GPU run is
 * reported as the io::Error of the chunk (pipeline.rs:163, :408-414). */
int blt_bpe_clear_error(const blt_bpe *h);

/* Number of distinct map entries; *single_pass = 1 when one greedy pass is provably the
 * fixpoint (no map value is a key component: true for every merges file below 65 281 lines). */
int blt_bpe_info(const blt_bpe *h, size_t *n_entries, int *single_pass);

/* ---------------------------------------------------------------------------------------
 * Host-buffer entry points (stage through the GPU; results are bit-exact with the reference).
 * ------------------------------------------------------------------------------------- */

/* TokenizationStrategy::process_chunk for BpeStrategy (tokenizer.rs:56-93): one chunk ->
 * big-endian u16 tokens.  out_cap must be >= 2 * n.  Empty input -> *out_len = 0. */
int blt_bpe_process_chunk(const blt_bpe *h, const uint8_t *in, size_t n, uint8_t *out, size_t out_cap,
                          size_t *out_len);

/* The mmap pipeline for a BPE strategy (pipeline.rs:56-192): split in into chunks of
 * chunk_size bytes (pipeline.rs:73-81), tokenise each chunk independently, concatenate in chunk
 * order.  Windows of whole chunks are dealt round-robin over min(n_gpus, visible devices)
 * devices (no collective); per device one thread copies windows in and launches their merge
 * scans while another copies each window's tokens straight to its final offset in out as soon as
 * every earlier window is counted, so devices overlap and nothing packs the output afterwards.
 * The output is identical for every n_gpus.  chunk_out_len (nullable) receives each chunk's
 * output bytes.  out_cap >= 2 * n. */
int blt_bpe_process_chunks(const blt_bpe *h, const uint8_t *in, size_t n, size_t chunk_size, int n_gpus,
                           uint8_t *out, size_t out_cap, size_t *out_len, uint64_t *chunk_out_len);

/* BasicTokenizationStrategy::process_chunk (tokenizer.rs:103-124): byte b -> [0, b]. */
int blt_basic_process_chunk(const uint8_t *in, size_t n, uint8_t *out, size_t out_cap, size_t *out_len);

/* run_tokenizer (lib.rs:246-267) with its pipeline (pipeline.rs:22-433): input file (mmap, fixed
 * chunks, pipeline.rs:73-81) or stdin (one read per chunk, at most min(chunk_size, 2 MiB) bytes as
 * tokio's stdin reads), the content-type token, every chunk through the selected strategy
 * (lib.rs:271-282: passthrough > bpe > basic) and the outputs in chunk order to the output file
 * (created and truncated after the input is opened, io_handler.rs:55-78) or stdout.  threads and
 * chunk_size are CoreConfig's resolved values (blt_determine_thread_count,
 * blt_effective_chunk_size).  Errors are the reference's io::Error texts ("No such file or
 * directory (os error 2)", ...) with their BLT_E_* kind; the first error of a run is returned. */
typedef struct blt_run_config {
    const char *input_path;   /* NULL: stdin */
    const char *output_path;  /* NULL: stdout */
    const blt_bpe *bpe;       /* BPE strategy, or NULL for the basic strategy */
    int passthrough;          /* nonzero: PassthroughStrategy (wins over bpe) */
    uint32_t content_token;   /* 0: none, else BLT_CONTENT_* written big-endian first */
    uint64_t threads;         /* chunks in flight (CoreConfig::num_threads, >= 1) */
    uint64_t chunk_size;      /* effective chunk size in bytes (> 0) */
    int n_gpus;               /* devices the file path shards each window over; 0 = all visible */
} blt_run_config;

int blt_run_tokenizer(const blt_run_config *cfg);

/* Logging of run_tokenizer, as the reference binary sets it up (src/main.rs:83-85:
 * tracing_subscriber::fmt with the RUST_LOG env filter): reads RUST_LOG (BLT_LOG when RUST_LOG is
 * unset) once; without either only errors are logged.  Lines go to stdout, as tracing's fmt
 * subscriber writes them: "<UTC time>  LEVEL <target>: <message> <field>=<value>".  Messages and
 * levels follow the reference: lib.rs:247, :251, :265, :273-279 (info), pipeline.rs:63, :203 (info),
 * pipeline.rs:108, :315, :323, :401 (debug, per chunk), pipeline.rs:409 (error), tokenizer.rs:113
 * (debug).  A library user that does not call it (the Python binding, as blt_python) logs nothing. */
void blt_log_init_from_env(void);

/* ---------------------------------------------------------------------------------------
 * Device-resident entry points (inputs already in HBM on the current HIP device).
 * ------------------------------------------------------------------------------------- */

/* Bytes of scratch workspace blt_bpe_encode_device needs for n input bytes.  Depends on the map:
 * a cyclic general map (a value that can be made from itself, below 2^32 input bytes) adds about
 * 1.8 n bytes for its sparse passes (bitmaps, seed and merge lists, compaction words). */
size_t blt_bpe_workspace_size(const blt_bpe *h, uint64_t n, uint64_t chunk_size);

/* Whole-buffer BPE over chunks of chunk_size bytes, on the current device and the given HIP
 * stream (NULL = default stream).  Fails with BLT_E_IO while the handle has a sticky device error
 * (blt_bpe_clear_error).  d_in: n bytes, 16-byte aligned.  d_out: 2 * n bytes,
 * 16-byte aligned; receives the stitched big-endian token stream.  d_chunk_off (nullable):
 * nchunks + 1 u64, the output token index where each chunk starts, [nchunks] = total tokens.
 * d_workspace: blt_bpe_workspace_size() bytes.  out_tokens (nullable): if given, the call
 * waits for the stream and returns the number of output tokens; if NULL, the call only enqueues
 * work (no host synchronisation) for every single-pass map and for every general map whose merge
 * chains are bounded (no value can be made from itself: its passes are known up front).  A
 * general map with a cycle (e.g. (97, 98) -> 97) waits for the stream after its first u16 pass
 * and then after every 4, to read whether the chain has reached its fixpoint.  A general map whose
 * bucket table fits in LDS (and that has a key with a token component) runs its first two passes
 * in one kernel whenever the call waits anyway (out_tokens given, or a cyclic map), falling back
 * to two kernels for input the fused kernel cannot resolve; the output is the same either way. */
int blt_bpe_encode_device(const blt_bpe *h, const uint8_t *d_in, uint64_t n, uint64_t chunk_size,
                          uint8_t *d_out, uint64_t *d_chunk_off, void *d_workspace, size_t workspace_bytes,
                          void *stream, uint64_t *out_tokens);

/* Flags of blt_bpe_encode_device_ex. */
#define BLT_ENCODE_WORKSPACE_ZEROED 1u /* the workspace's look-back words are zero: the caller ran
                                          blt_bpe_workspace_reset on this stream for an n at least this
                                          call's since the last encode, or the last encodes on it were
                                          single-pass ones (single-pass maps; ignored otherwise) */

/* As blt_bpe_encode_device, with flags.  With BLT_ENCODE_WORKSPACE_ZEROED the call enqueues only
 * the merge-scan kernel, so events around it time that kernel alone.  A single-pass encode leaves
 * the workspace's ticket and status words zeroed when its kernel ends (its last workgroup resets
 * them), so back-to-back single-pass encodes on one stream and workspace need one reset before the
 * first only; the error flags stay until blt_bpe_check_workspace or a reset.  The control block
 * records how many status words are known zero (word 14: set by blt_bpe_workspace_reset to its
 * n's tile count, raised by each single-pass kernel's self-reset to its own, cleared by a general
 * map's passes and by blt_bpe_check_workspace after an error).  A flagged launch needing more
 * words than that refuses: it writes nothing and flags error bit 32, which the next
 * blt_bpe_check_workspace reports and which fails the handle's next call (BLT_E_IO) until
 * blt_bpe_clear_error.  Reset for the largest n encoded with the flag. */
int blt_bpe_encode_device_ex(const blt_bpe *h, const uint8_t *d_in, uint64_t n, uint64_t chunk_size,
                             uint8_t *d_out, uint64_t *d_chunk_off, void *d_workspace, size_t workspace_bytes,
                             void *stream, uint64_t *out_tokens, uint32_t flags);

/* Enqueues the zeroing of the look-back control words an encode of (n, chunk_size) uses. */
int blt_bpe_workspace_reset(const blt_bpe *h, void *d_workspace, uint64_t n, uint64_t chunk_size, void *stream);

/* Reads and clears the device error flags a previous async encode left in d_workspace
 * (waits for the stream).  0 if clean, BLT_E_IO if a look-back timed out or a range or prefix
 * check failed.  (The handle's sticky error, blt_bpe_clear_error, is separate.) */
int blt_bpe_check_workspace(void *d_workspace, void *stream);

/* Basic strategy on device: d_out[2i] = 0, d_out[2i + 1] = d_in[i]. */
int blt_basic_encode_device(const uint8_t *d_in, uint64_t n, uint8_t *d_out, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* BLT_BPE_H */
