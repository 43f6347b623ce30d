// Grouped fp16 MFMA GEMM (include/s3n.h s3n_gemm): argument checks and the
// C ABI.  The kernel template is net_gemm_kernel.hpp; its tile families are
// instantiated in net_gemm_t1..t5.hip, the halo conv in net_gemm_t6.hip, the
// B-direct tiles in net_gemm_t9.hip (compiled in parallel).
#include "net_gemm_kernel.hpp"

namespace s3gemm {
int g_xcd_flags = 0;
}  // namespace s3gemm

static int g_gemm_debug = 0;

int s3n_ln_f16_saturations(int reset);   // net_ops.hip

extern "C" int s3n_f16_saturations(int reset) {
  int any = 0;
  for (auto fn : {s3gemm::sat_t1, s3gemm::sat_t2, s3gemm::sat_t3, s3gemm::sat_t4, s3gemm::sat_t5,
                  s3gemm::sat_t6, s3gemm::sat_t7, s3gemm::sat_t8, s3gemm::sat_t9}) {
    const int v = fn(reset);
    if (v < 0) return -1;
    any |= v;
  }
  const int l = s3n_ln_f16_saturations(reset);
  if (l < 0) return -1;
  return any + l;
}
extern "C" void s3n_gemm_set_debug(int flags) { g_gemm_debug = flags; }
extern "C" void s3n_gemm_set_xcd_flags(int flags) { s3gemm::g_xcd_flags = flags; }

extern "C" size_t s3n_gemm_workspace_bytes(const s3n_gemm_args* a) {
  if (!a || a->split_k <= 1) return 0;
  return sizeof(float) * (size_t)a->groups * a->split_k * (size_t)a->M * a->N;
}

extern "C" int s3n_gemm(const s3n_gemm_args* a, void* stream) {
  S3_REQUIRE(a && a->M >= 0 && a->N > 0 && a->K > 0, "s3n_gemm: bad sizes");
  S3_REQUIRE(a->groups >= 1 && a->groups <= S3N_MAX_GROUPS, "s3n_gemm: groups must be 1..4");
  S3_REQUIRE(a->K % 8 == 0, "s3n_gemm: K must be a multiple of 8 (16-B operand chunks)");
  if (a->a_mode == S3N_A_DENSE) S3_REQUIRE(a->lda % 8 == 0, "s3n_gemm: lda %% 8 != 0");
  S3_REQUIRE(a->ldb % 8 == 0, "s3n_gemm: ldb %% 8 != 0");
  if (a->a_mode == S3N_A_CONV) {
    S3_REQUIRE(a->cC % 8 == 0, "s3n_gemm: conv Cin must be a multiple of 8");
    S3_REQUIRE(a->K == a->ksize * a->ksize * a->cC, "s3n_gemm: conv K != ks*ks*Cin");
    S3_REQUIRE(a->oH > 0 && a->oW > 0 && a->M % (a->oH * a->oW) == 0, "s3n_gemm: conv M");
  }
  const bool tail = a->tail_w[0] != nullptr;
  for (int g = 0; g < a->groups; ++g)
    S3_REQUIRE(a->A[g] && a->B[g] && (a->C[g] || tail) && (!tail || (a->tail_w[g] && a->tail_out[g])),
               "s3n_gemm: null operand in group %d", g);
  if (tail)
    S3_REQUIRE(a->tail_n > 0 && a->tail_n % 8 == 0 && a->tail_n <= 16 && a->ld_tail % 8 == 0 &&
                   a->split_k <= 1 && a->store_mode == S3N_STORE_PLAIN,
               "s3n_gemm: tail needs tail_n in {8, 16}, ld_tail %% 8 == 0, split_k 1, plain store");
  if (a->M == 0) return S3_OK;
  GemmP p;
  p.M = a->M; p.N = a->N; p.K = a->K; p.groups = a->groups;
  for (int g = 0; g < S3N_MAX_GROUPS; ++g) {
    const bool on = g < a->groups;
    p.A[g] = on ? (const f16*)a->A[g] : nullptr;
    p.B[g] = on ? (const f16*)a->B[g] : nullptr;
    p.bias[g] = on ? a->bias[g] : nullptr;
    p.R1[g] = on ? a->R1[g] : nullptr;
    p.R2[g] = on ? a->R2[g] : nullptr;
    p.C[g] = on ? a->C[g] : nullptr;
    p.C2[g] = on ? (f16*)a->C2[g] : nullptr;
    p.Bp[g] = on ? (const f16*)a->Bp[g] : nullptr;
  }
  p.lda = a->lda; p.ldb = a->ldb; p.ldr1 = a->ldr1; p.r1_f16 = a->r1_f16;
  p.ldr2 = a->ldr2; p.r2_f16 = a->r2_f16; p.ldc = a->ldc; p.c_f16 = a->c_f16;
  p.ldc2 = a->ldc2; p.act = a->act; p.store_mode = a->store_mode; p.a_mode = a->a_mode;
  p.cH = a->cH; p.cW = a->cW; p.cC = a->cC; p.ks = a->ksize; p.st = a->stride; p.pad = a->pad;
  p.oH = a->oH; p.oW = a->oW; p.relu_in = a->relu_in;
  p.sH = a->sH; p.sW = a->sW; p.sS = a->sS; p.sCout = a->sCout;
  p.split_k = a->split_k > 1 ? a->split_k : 1;
  p.rope_cos = a->rope_cos;
  p.rope_sin = a->rope_sin;
  p.rope_ncols = a->rope_ncols;
  bool any_rope = false;
  for (int g = 0; g < S3N_MAX_GROUPS; ++g) {
    p.rope_pos[g] = g < a->groups ? a->rope_pos[g] : nullptr;
    any_rope = any_rope || p.rope_pos[g];
  }
  if (any_rope) {
    S3_REQUIRE(p.split_k == 1 && a->rope_cos && a->rope_sin && a->rope_ncols % 64 == 0 &&
                   a->rope_ncols <= a->N && a->store_mode == S3N_STORE_PLAIN,
               "s3n_gemm: RoPE epilogue needs split_k 1, tables, ncols %% 64 == 0, plain store");
    for (int g = 0; g < a->groups; ++g)
      S3_REQUIRE(a->rope_pos[g], "s3n_gemm: RoPE positions missing for group %d", g);
  }
  p.ws = static_cast<float*>(a->workspace);
  p.debug = g_gemm_debug;
  // 8-column vector epilogue: every row stride a multiple of 8 elements,
  // every base 16-B aligned, chunks contiguous in the output layout
  {
    auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    bool v = a->N % 8 == 0 && (!(g_gemm_debug & 16) || tail);
    if (a->store_mode == S3N_STORE_PLAIN) v = v && a->ldc % 8 == 0;
    else if (a->store_mode == S3N_STORE_CONVT) v = v && a->sCout % 8 == 0;
    else v = false;
    for (int g = 0; g < a->groups && v; ++g) {
      v = (!a->C[g] || al(a->C[g])) && (!a->bias[g] || al(a->bias[g])) &&
          (!a->tail_w[g] || (al(a->tail_w[g]) && al(a->tail_out[g]) &&
                             (!a->tail_b[g] || al(a->tail_b[g])))) &&
          (!a->R1[g] || (al(a->R1[g]) && a->ldr1 % 8 == 0)) &&
          (!a->R2[g] || (al(a->R2[g]) && a->ldr2 % 8 == 0)) &&
          (!a->C2[g] || (al(a->C2[g]) && a->ldc2 % 8 == 0));
    }
    if (any_rope) v = v && al(a->rope_cos) && al(a->rope_sin);
    p.vec_epi = v ? 1 : 0;
    S3_REQUIRE(!tail || v, "s3n_gemm: the fused tail needs the vector epilogue (aligned operands, "
                           "N %% 8 == 0)");
  }
  for (int g = 0; g < S3N_MAX_GROUPS; ++g) {
    const bool on = g < a->groups && tail;
    p.tail_w[g] = on ? (const f16*)a->tail_w[g] : nullptr;
    p.tail_b[g] = on ? a->tail_b[g] : nullptr;
    p.tail_out[g] = on ? a->tail_out[g] : nullptr;
  }
  p.tail_n = a->tail_n;
  p.ld_tail = a->ld_tail;
  if (p.split_k > 1)
    S3_REQUIRE(p.ws, "s3n_gemm: split_k > 1 needs a workspace (s3n_gemm_workspace_bytes)");
  hipStream_t st = s3::as_stream(stream);
  // tile families live in their own translation units (net_gemm_t*.hip)
  for (auto fn : {s3gemm::launch_t1, s3gemm::launch_t2, s3gemm::launch_t3, s3gemm::launch_t4,
                  s3gemm::launch_t5, s3gemm::launch_t6, s3gemm::launch_t7,
                  s3gemm::launch_t8, s3gemm::launch_t9}) {
    const int r = fn(a->tile, p, st);
    if (r != s3gemm::kNotMine) return r;
  }
  S3_REQUIRE(false, "s3n_gemm: unknown tile %d", a->tile);
}
