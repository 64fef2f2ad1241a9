/* A plain-C consumer of include/okvisgpu.h (C99, -pedantic): proves the header is a C ABI (no C++
 * or HIP types) and drives one solve through it, the way a cgo / JNI / ctypes stub would bind it.
 * Usage: abi_consumer cpu   (no GPU: version, options, generator, error paths)
 *        abi_consumer gpu   (S10 synthetic window: set_problems + solve, prints the summary) */
#include <stdio.h>
#include <string.h>

#include "okvisgpu.h"

static int fail(const char* what, int rc) {
  fprintf(stderr, "abi_consumer: %s failed (%d): %s\n", what, rc, okvisgpu_last_error(NULL));
  return 1;
}

int main(int argc, char** argv) {
  const int gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
  okvisgpu_options o;
  okvisgpu_synth_config cfg;
  okvisgpu_synth_window* w = NULL;
  const okvisgpu_problem* p;
  okvisgpu_ctx* ctx = NULL;
  okvisgpu_summary s;
  int rc;
  if (okvisgpu_abi_version() != OKVISGPU_ABI_VERSION) return fail("abi_version", okvisgpu_abi_version());
  okvisgpu_default_options(&o);
  if (o.linear_solver != OKVISGPU_DENSE_SCHUR || o.trust_region_strategy != OKVISGPU_DOGLEG) return fail("defaults", 0);
  okvisgpu_synth_default_config(&cfg, 10, 500, 4000, 20251015u);
  rc = okvisgpu_synth_create(&cfg, &w);
  if (rc != OKVISGPU_OK) return fail("synth_create", rc);
  p = okvisgpu_synth_problem(w);
  if (p->n_poses != 10 || p->n_landmarks != 500 || p->n_observations != 4000) return fail("synth sizes", 0);
  if (!gpu) {
    rc = okvisgpu_solve(NULL, &o, &s);
    if (rc != OKVISGPU_ERR_INVALID_ARGUMENT) return fail("solve(NULL) must be rejected", rc);
    printf("abi_consumer cpu ok: ABI %d, %d poses / %d landmarks / %d observations\n", okvisgpu_abi_version(),
           p->n_poses, p->n_landmarks, p->n_observations);
    okvisgpu_synth_destroy(w);
    return 0;
  }
  rc = okvisgpu_ctx_create(0, &ctx);
  if (rc != OKVISGPU_OK) return fail("ctx_create", rc);
  rc = okvisgpu_set_problems(ctx, p, 1);
  if (rc != OKVISGPU_OK) return fail("set_problems", rc);
  o.max_num_iterations = 10;
  rc = okvisgpu_solve(ctx, &o, &s);
  if (rc != OKVISGPU_OK) return fail("solve", rc);
  printf("{\"initial_cost\": %.17g, \"final_cost\": %.17g, \"num_iterations\": %d, \"termination\": %d, "
         "\"pose9\": [%.17g, %.17g, %.17g]}\n",
         s.initial_cost, s.final_cost, s.num_iterations, s.termination_type, p->poses[63], p->poses[64], p->poses[65]);
  okvisgpu_ctx_destroy(ctx);
  okvisgpu_synth_destroy(w);
  return 0;
}
