// rs_jit.hpp — bit-sliced GF(2)-linear network kernels, generated per plan and
// compiled at plan time with hipRTC for gfx950.
//
// Both codec operations are, per 16-bit symbol position, GF(2)-linear maps from
// the shards read to the shards written (encode: k data -> m parity,
// root.zig:136-173; reconstruct for one erasure pattern: k received -> e
// restored, root.zig:268-335; SURVEY.md §A.6 column independence). A plan turns
// that map into a (16*n_out) x (16*n_in) GF(2) matrix and emits a kernel whose
// lanes hold 32 symbols per shard as 16 bit-planes (one dword per bit position,
// three delta-swap stages of a byte-lane 8x8 bit transpose on the way in and
// out) and evaluate the matrix as a straight-line XOR network of v_bitop3_b32
// (XOR3, full rate on gfx950). The matrix is a compile-time constant of the
// generated source, so the network carries no table reads and no v_perm_b32
// (half rate), which is what bounds the table-driven kernels in rs_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <sstream>
#include <string>
#include <vector>

namespace rs {
namespace jit {

// One network: out[j] = XOR_t M_jt(in[t]) over n_in input shards.
//   src[t]  : input shard t = (src & kSrcRecovery ? buffer 1 : buffer 0)[src & kSrcIndexMask]
//   images  : images[(t * n_out + j) * 16 + b] = M_jt(1 << b) (16-bit symbol images)
struct NetSpec {
  std::string role = "net";  // "encode" / "reconstruct": kernel symbol rs_net_<role>_i<n_in>_o<n_out>_<hash>
  uint32_t n_in = 0, n_out = 0;
  std::vector<int32_t> src;
  std::vector<uint16_t> images;
  // stripes per 4 KiB wave unit: 1 (shards of whole 4 KiB units), or 2 / 4 for
  // 2 KiB / 1 KiB shards, where a wave's four 1 KiB pieces come from that many
  // consecutive stripes (chosen per launch from the shard size, net_pieces)
  uint32_t pieces = 1;
};

// Lanes cover 4 KiB of every shard per wave (32 symbols per lane): shard_bytes
// must be a multiple of this (or 1 / 2 KiB, NetSpec::pieces), below 4 GiB.
constexpr uint64_t kUnitBytes = 4096;
constexpr uint32_t kTileOut = 4;      // size caps count blocks of one input x 4 outputs
constexpr uint32_t kMaxOut = 64;      // tiles of 8 outputs (RS_AMD_NET_TILE), one workgroup each
// generated code size: n_in x tiles input blocks of ~270 instructions each; hipRTC
// takes ~20-40 ms per block, so the cap keeps a plan's compile near 1-2 s
// (max_blocks())
constexpr uint64_t kMaxBlocks = 64;
uint64_t max_blocks();
// Larger maps (the e x e syndrome map of wide codes: RS(200,55) losing 55 is 770
// blocks, ~16-36 s) compile in a background thread while the plan's table kernel
// runs; RS_AMD_NET_ASYNC_BLOCKS overrides the cap (0 = never), RS_AMD_JIT_SYNC=1
// compiles them in the calling thread instead.
constexpr uint64_t kMaxAsyncBlocks = 1024;
uint64_t max_async_blocks();
bool supports_async(uint32_t n_in, uint32_t n_out, uint64_t shard_bytes);

// shard sizes the networks cover: whole 4 KiB units below 4 GiB (32-bit lane
// offsets), or 1 KiB / 2 KiB shards (a wave unit then spans 4 / 2 stripes)
bool shard_ok(uint64_t shard_bytes);
uint32_t net_pieces(uint64_t shard_bytes);  // NetSpec::pieces for this shard size

bool enabled();  // RS_AMD_JIT != 0 and hipRTC usable
bool supports(uint32_t n_in, uint32_t n_out, uint64_t shard_bytes);

// CUDA-style source of the kernel `name` (exposed for tests / inspection).
std::string generate(const NetSpec &spec, const std::string &name);

// Building blocks for other generated kernels: the device prelude (tr8 / ld / planes /
// st over a wave's 4 KiB unit; RS_NT must be defined first), and one input's
// Four-Russians XOR network into accumulators a<r> (rows[r] = 16-bit mask of the
// input planes feeding accumulator r; `init`: accumulators already assigned).
std::string net_prelude();  // RS_AMD_NET_VMASK (default 1): transpose masks in VGPRs
bool net_vmask();
void emit_network_input(std::ostringstream &o, const std::vector<uint16_t> &rows, std::vector<bool> &init, int t);

struct Kernel {
  hipModule_t module = nullptr;
  hipFunction_t fn = nullptr;
  uint32_t n_in = 0, n_out = 0, n_tiles = 0, units = 1, pieces = 1;
  bool shared = false;  // shared-input form: one workgroup of n_tiles waves per 4 KiB unit
  std::string name;
  double compile_ms = 0;
};

// Compiled kernel for `spec` on the current device (cached by content). Returns
// nullptr and sets `err` when hipRTC is unavailable or compilation fails.
const Kernel *get(const NetSpec &spec, std::string &err);

// Same, for maps past the synchronous cap: returns the kernel once compiled; until
// then nullptr with pending = true (a background compile has been started), or
// nullptr with pending = false and `err` set if the compile failed.
const Kernel *get_async(const NetSpec &spec, std::string &err, bool &pending);

// Any generated kernel: `gen` returns a complete source defining extern "C" `name`;
// compiled once per (device, key). async: compiled on the background worker
// (nullptr + pending until it is loaded; RS_AMD_JIT_SYNC=1 compiles in the caller).
const Kernel *get_source(const std::string &key, const std::string &name, const std::function<std::string()> &gen,
                         bool async, std::string &err, bool &pending);
// hipRTC compile of a source only (no device): a build check.
bool compile_source_check(const std::string &src, std::string &err, double *ms, size_t *code_bytes);

// hipRTC compiles run, code objects found in the disk cache, modules loaded (this process)
void compile_stats(uint64_t *compiles, uint64_t *disk_hits, uint64_t *modules);

// Block until no background compile or host job is running (rs_net_wait).
void wait_pending();
// compiles and host jobs queued or running on the background worker
size_t pending_jobs();
// Run `fn` on the background worker, in order with the compiles (the current device set),
// once per key while pending; false if the worker is unavailable. At exit the queue is
// dropped and a running job finishes before the HIP runtime's teardown (as a compile).
bool run_host_job(const std::string &key, std::function<void()> fn);

// Generate and compile `spec` with hipRTC only (no device needed): a build check.
bool compile_check(const NetSpec &spec, std::string &err, double *ms, size_t *code_bytes);

// buf0/buf1: input buffers ([stripe][shard][sb]); out: [stripe][n_out][sb]. An input
// flagged kSrcXorScratch is buf1[idx] ^ buf2[idx] (buf2: [stripe][..][sb], stride2).
hipError_t launch(const Kernel &k, const uint8_t *buf0, uint64_t stride0, const uint8_t *buf1, uint64_t stride1,
                  uint8_t *out, uint64_t out_stride, uint64_t shard_bytes, uint64_t n_stripes, hipStream_t s,
                  const uint8_t *buf2 = nullptr, uint64_t stride2 = 0);

}  // namespace jit
}  // namespace rs
