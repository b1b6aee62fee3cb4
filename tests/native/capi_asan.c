/* Host-side checks of liblic's C ABI under AddressSanitizer (CPU only, no GPU needed).
 * Built against liblic_asan.so (csrc/Makefile target `asan`: host code compiled with
 * -fsanitize=address, no device code) by tests/test_capi_asan.py.  Exercises every
 * host-only helper and the argument validation of the launch entry points (they must
 * fail with a message, never dereference a bad argument), and the thread-local
 * lic_last_error from 8 threads at once.  Prints CAPI_OK on success.            */
#include <pthread.h>
#include <stdio.h>
#include <string.h>

#include "lic.h"

static int nfail = 0;
#define EXPECT_FAIL(call, substr)                                                          \
  do {                                                                                     \
    int r_ = (call);                                                                       \
    if (r_ == 0 || !strstr(lic_last_error(), substr)) {                                   \
      fprintf(stderr, "FAIL %s: status %d, error '%s' (want '%s')\n", #call, r_, lic_last_error(), substr); \
      ++nfail;                                                                             \
    }                                                                                      \
  } while (0)
#define EXPECT(cond)                                           \
  do {                                                         \
    if (!(cond)) {                                             \
      fprintf(stderr, "FAIL %s (line %d)\n", #cond, __LINE__); \
      ++nfail;                                                 \
    }                                                          \
  } while (0)

static void* worker(void* arg) {
  const long id = (long)arg;
  char want[64];
  for (int i = 0; i < 2000; ++i) {
    lic_conv_args a;
    memset(&a, 0, sizeof a);
    a.ntaps = (id & 1) ? 0 : LIC_MAX_TAPS + 1 + (int)id;   /* "ntaps out of range" */
    if (lic_conv2d_fwd(&a, 0) == 0) return (void*)1;
    snprintf(want, sizeof want, "ntaps");
    if (!strstr(lic_last_error(), want)) return (void*)2;
    lic_attn_args t;
    memset(&t, 0, sizeof t);
    if (lic_win_attn_fwd(&t, 0) == 0 || !strstr(lic_last_error(), "attn")) return (void*)3;
  }
  return NULL;
}

int main(void) {
  /* host-only helpers */
  EXPECT(lic_rans_cap(256) > 0 && lic_rans_cap(4096) > lic_rans_cap(256));
  EXPECT(lic_lam_parts(4) > 0);
  EXPECT(lic_channel_sum_workspace(192) > 0);
  EXPECT(lic_layernorm_bwd_workspace(4096, 128) > 0);
  EXPECT(lic_dwconv_wgrad_workspace(2, 16, 16, 64, 9) > 0);
  EXPECT(lic_rate_train_parts(4096, 48) > 0);
  EXPECT(lic_recon_train_blocks(65536) > 0);
  EXPECT(strstr(lic_version(), "gfx950") != NULL);

  /* struct entry points: NULL and inconsistent arguments */
  EXPECT_FAIL(lic_conv2d_fwd(NULL, 0), "null");
  lic_conv_args c;
  memset(&c, 0, sizeof c);
  EXPECT_FAIL(lic_conv2d_fwd(&c, 0), "ntaps");
  c.ntaps = LIC_MAX_TAPS + 1;
  EXPECT_FAIL(lic_conv2d_fwd(&c, 0), "ntaps");
  EXPECT_FAIL(lic_win_attn_fwd(NULL, 0), "null");
  lic_attn_args at;
  memset(&at, 0, sizeof at);
  static float dummy[64];
  at.qkv = dummy; at.out = dummy; at.table = dummy; at.c = 8; at.heads = 3;
  EXPECT_FAIL(lic_win_attn_fwd(&at, 0), "heads");
  EXPECT_FAIL(lic_gauss_rate_fwd(NULL, 0), "null");
  EXPECT_FAIL(lic_rans_encode(NULL, 0), "null");
  EXPECT_FAIL(lic_rans_decode(NULL, 0), "null");
  lic_rans_args ra;
  memset(&ra, 0, sizeof ra);
  static int32_t idummy[64];
  static uint32_t udummy[64];
  ra.n = 1; ra.hw = 4; ra.c = 2; ra.ctot = 2; ra.c0 = 1;
  ra.symbols = idummy; ra.cdfs = idummy; ra.cdf_sizes = idummy; ra.offsets = idummy;
  ra.scratch = udummy; ra.lengths = idummy; ra.cap = lic_rans_cap(4);
  EXPECT_FAIL(lic_rans_encode(&ra, 0), "channel window");
  ra.c0 = 0; ra.cap = 1;
  EXPECT_FAIL(lic_rans_encode(&ra, 0), "lic_rans_cap");
  ra.words = udummy; ra.offsets_w = udummy; ra.c0 = 1;
  EXPECT_FAIL(lic_rans_decode(&ra, 0), "channel window");
  EXPECT(lic_conv2d_wgrad_workspace(NULL) == -1);
  EXPECT_FAIL(lic_conv2d_wgrad(NULL, 0), "null");
  EXPECT(lic_win_attn_bwd_workspace(NULL) == -1);
  EXPECT_FAIL(lic_win_attn_bwd(NULL, dummy, 0, dummy, 0, dummy, 0, dummy, 0, 0), "null");
  EXPECT_FAIL(lic_pmf_to_cdf(dummy, idummy, 1, 4, 0, idummy, 4, idummy, 0), "precision");
  EXPECT_FAIL(lic_gdn_prepare(LIC_F32, dummy, dummy, 16, 0.f, 0.f, 0.f, dummy, 8, 16, dummy, 0), "padding");
  EXPECT_FAIL(lic_channel_sum(LIC_F32, dummy, 16, 4, 16, dummy, 1, dummy, 0, 0), "workspace");

  /* thread-local error state */
  pthread_t th[8];
  for (long i = 0; i < 8; ++i) pthread_create(&th[i], NULL, worker, (void*)i);
  for (int i = 0; i < 8; ++i) {
    void* r = NULL;
    pthread_join(th[i], &r);
    if (r) {
      fprintf(stderr, "FAIL thread %d: code %ld\n", i, (long)r);
      ++nfail;
    }
  }
  if (nfail) return 1;
  printf("CAPI_OK\n");
  return 0;
}
