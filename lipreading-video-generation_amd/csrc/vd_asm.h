// vd_asm.h -- argument blocks and launchers of the hand-scheduled kernels
// (asm/gen_attn_asm.py; asm_kernels.cpp).  Internal to libvdiff.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vd {

// vd_attn_bwd_dq_d64 kernarg block (gen_attn_asm.py KARG layout, 128 bytes).  Byte
// quantities are offsets from the sequence base; *_bytes ranges bound the buffer range
// checks that zero-fill rows past the sequence end.
struct AsmDqArgs {
  const void* q;
  const void* k;
  const void* v;
  const void* dout;
  const float* nlse2;
  const float* ndelta;
  void* dq;
  uint32_t n, ts_bytes, ots_bytes, groups;
  uint64_t bs_bytes, gs_bytes, obs_bytes, ogs_bytes;
  float scale, qscale;
  uint32_t kv_bytes, o_bytes, tile_bytes, niter;
};
static_assert(sizeof(AsmDqArgs) == 128, "kernarg block layout");

// grid (ceil(n / 256), groups, nseq / groups), 256 threads, 64 KiB static LDS
int asm_bwd_dq_d64(const AsmDqArgs& a, unsigned gx, unsigned gy, unsigned gz,
                   hipStream_t stream);

// vd_attn_bwd_dkdv_d64 kernarg block (gen_attn_asm.py dK/dV layout, 144 bytes)
struct AsmDkdvArgs {
  const void* q;
  const void* k;
  const void* v;
  const void* dout;
  const float* nlse2;
  const float* ndelta;
  void* dk;
  void* dv;
  uint32_t n, ts_bytes, ots_bytes, groups;
  uint64_t bs_bytes, gs_bytes, obs_bytes, ogs_bytes;
  float scale, kscale;
  uint32_t kv_bytes, o_bytes, tile_bytes, otile_bytes, niter, pad;
};
static_assert(sizeof(AsmDkdvArgs) == 144, "kernarg block layout");

// grid (ceil(n / 256), groups, nseq / groups), 256 threads, 67 KiB static LDS
int asm_bwd_dkdv_d64(const AsmDkdvArgs& a, unsigned gx, unsigned gy, unsigned gz,
                     hipStream_t stream);

// vd_attn_bwd_dq_d128 (asm/gen_d128.py): the dQ kernarg block; grid (ceil(n / 128), groups,
// nseq / groups), 256 threads, 128 KiB static LDS
int asm_bwd_dq_d128(const AsmDqArgs& a, unsigned gx, unsigned gy, unsigned gz,
                    hipStream_t stream);

// vd_attn_bwd_dkdv_d128 (asm/gen_d128.py): the same kernarg block; grid (ceil(n / 128),
// groups, nseq / groups), 256 threads, 131 KiB static LDS
int asm_bwd_dkdv_d128(const AsmDkdvArgs& a, unsigned gx, unsigned gy, unsigned gz,
                      hipStream_t stream);

// vd_attn_fwd_d64 kernarg block (asm/gen_fwd.py, 112 bytes): niter = 512-key iterations
// (the last one masks keys >= n), klim0 = keys in the last iteration
struct AsmFwdArgs {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  float* lse;
  uint32_t n, ts_bytes, ots_bytes, groups;
  uint64_t bs_bytes, gs_bytes, obs_bytes, ogs_bytes;
  float qscale;
  uint32_t kv_bytes, o_bytes, tile_bytes, niter, klim0;
};
static_assert(sizeof(AsmFwdArgs) == 112, "kernarg block layout");

// grid (ceil(n / 256), groups, nseq / groups), 256 threads, 128 KiB static LDS
int asm_fwd_d64(const AsmFwdArgs& a, unsigned gx, unsigned gy, unsigned gz, hipStream_t stream);

// vd_attn_fwd_d128 (asm/gen_fwd128.py): the same block with 32-row tiles (tile_bytes, niter
// = 256-key iterations, klim0); grid (ceil(n / 256), groups, nseq / groups), 128 KiB LDS
int asm_fwd_d128(const AsmFwdArgs& a, unsigned gx, unsigned gy, unsigned gz, hipStream_t stream);

// vd_attn_bwd_dq_d256 (asm/gen_d256.py): the dQ block plus the key split -- split z of
// 2^lsplit takes keys [z kps, (z + 1) kps) and, with part != 0, writes dQ * scale as fp32
// partials part[z][seq][n][256] (split_bytes = nseq * n * 1024, part_bytes = n * 1024).
// grid (ceil(n / 128), groups, (nseq / groups) << lsplit), 256 threads, 128 KiB static LDS
struct AsmDq256Args {
  AsmDqArgs b;
  float* part;
  uint32_t kps, lsplit;
  uint64_t split_bytes;
  uint32_t part_bytes, pad;
};
static_assert(sizeof(AsmDq256Args) == 160, "kernarg block layout");
int asm_bwd_dq_d256(const AsmDq256Args& a, unsigned gx, unsigned gy, unsigned gz,
                    hipStream_t stream);

// vd_attn_bwd_dkdv_d256 (asm/gen_d256dk.py): the dK/dV block plus the query split -- split z
// of 2^lsplit takes queries [z qps, (z + 1) qps) and, with part != 0, writes fp32 partials
// part[z][seq][nkv][dK 256 | dV 256] (dK times scale; split_bytes = nseq * nkv * 2048,
// part_bytes = nkv * 2048).  tile_bytes / otile_bytes: 32 rows of q / dout.
// grid (ceil(n / 64), groups, (nseq / groups) << lsplit), 256 threads, 147 KiB static LDS
struct AsmDkdv256Args {
  AsmDkdvArgs b;
  float* part;
  uint32_t qps, lsplit;
  uint64_t split_bytes;
  uint32_t part_bytes, pad;
};
static_assert(sizeof(AsmDkdv256Args) == 176, "kernarg block layout");
int asm_bwd_dkdv_d256(const AsmDkdv256Args& a, unsigned gx, unsigned gy, unsigned gz,
                      hipStream_t stream);

// vd_attn_fwd_d256 (asm/gen_fwd256.py): the forward block plus the key split -- split z of
// 2^lsplit takes keys [z kps, min(n, (z + 1) kps)) and, with part != 0, writes its
// unnormalised O (fp32, part + z split_bytes: [seq][n][256]) and (m in log2 units, l) rows
// (part + ml_off + z ml_split_bytes: [seq][n][2]) in attention.hip's FwdSplit layout for
// attn_fwd_combine_kernel.  b.niter / b.klim0 are unused (the kernel derives its iterations
// from its split's key count).  grid (ceil(n / 128), groups, (nseq / groups) << lsplit), 256
// threads, 128 KiB static LDS
struct AsmFwd256Args {
  AsmFwdArgs b;
  float* part;
  uint32_t kps, lsplit;
  uint64_t split_bytes;
  uint64_t ml_off;
  uint32_t ml_split_bytes, pad[3];
};
static_assert(sizeof(AsmFwd256Args) == 160, "kernarg block layout");
int asm_fwd_d256(const AsmFwd256Args& a, unsigned gx, unsigned gy, unsigned gz,
                 hipStream_t stream);

}  // namespace vd
