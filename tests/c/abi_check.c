/* abi_check.c — a plain C99 client of include/karpenter_amd.h, compiled with gcc (no C++, no HIP
 * headers): what a cgo shim sees of the boundary.
 *
 *   abi_check inspect <snapshot.json>   host-only encode (no device): prints the layout JSON
 *   abi_check solve <snapshot.json>     ks_problem_create + ks_solve, then every structured accessor
 *                                       (ks_results_nodeclaim / _requests / _requirements /
 *                                       existing nodes / pod errors) printed as one JSON document
 *
 * tests/test_abi_c.py builds it and checks the solve output against ks_results_json's document. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "karpenter_amd.h"

static char* slurp(const char* path, size_t* len) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char* b = (char*)malloc((size_t)n + 1);
  if (!b || fread(b, 1, (size_t)n, f) != (size_t)n) {
    fclose(f);
    free(b);
    return NULL;
  }
  b[n] = 0;
  fclose(f);
  *len = (size_t)n;
  return b;
}

static void put_str(const char* s) {  /* JSON string (the boundary's strings are UTF-8 without controls) */
  putchar('"');
  for (; *s; s++) {
    if (*s == '"' || *s == '\\') putchar('\\');
    putchar(*s);
  }
  putchar('"');
}

static int fail(const char* what, int rc) {
  fprintf(stderr, "%s failed: %d %s\n", what, rc, ks_last_error());
  return 1;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s inspect|solve <snapshot.json>\n", argv[0]);
    return 2;
  }
  size_t len = 0;
  char* snap = slurp(argv[2], &len);
  if (!snap) {
    fprintf(stderr, "cannot read %s\n", argv[2]);
    return 2;
  }
  int rc;
  if (strcmp(argv[1], "inspect") == 0) {
    char* dims = NULL;
    if ((rc = ks_problem_inspect(snap, len, &dims)) != KS_OK) return fail("ks_problem_inspect", rc);
    printf("%s\n", dims);
    ks_free(dims);
    free(snap);
    return 0;
  }
  ks_problem* pb = NULL;
  if ((rc = ks_problem_create(snap, len, &pb)) != KS_OK) return fail("ks_problem_create", rc);
  ks_solve_opts opts;
  memset(&opts, 0, sizeof opts);
  opts.device = -1;
  opts.simulation_mode = 1;
  ks_results* r = NULL;
  if ((rc = ks_solve(pb, &opts, &r)) != KS_OK) return fail("ks_solve", rc);
  printf("{\"newNodeClaims\":[");
  int nc = ks_results_num_new_nodeclaims(r);
  for (int i = 0; i < nc; i++) {
    int tpl = -1, np = 0, nit = 0, nq = 0, nr = 0;
    const int32_t *pods = NULL, *its = NULL;
    const char *const *names = NULL, *const *qty = NULL;
    const ks_requirement* reqs = NULL;
    if ((rc = ks_results_nodeclaim(r, i, &tpl, &pods, &np, &its, &nit)) != KS_OK) return fail("ks_results_nodeclaim", rc);
    if ((rc = ks_results_nodeclaim_requests(r, i, &nq, &names, &qty)) != KS_OK) return fail("ks_results_nodeclaim_requests", rc);
    if ((rc = ks_results_nodeclaim_requirements(r, i, &nr, &reqs)) != KS_OK)
      return fail("ks_results_nodeclaim_requirements", rc);
    printf("%s{\"template\":%d,\"pods\":[", i ? "," : "", tpl);
    for (int k = 0; k < np; k++) printf("%s%d", k ? "," : "", pods[k]);
    printf("],\"instanceTypes\":[");
    for (int k = 0; k < nit; k++) printf("%s%d", k ? "," : "", its[k]);
    printf("],\"requests\":{");
    for (int k = 0; k < nq; k++) {
      if (k) putchar(',');
      put_str(names[k]);
      putchar(':');
      put_str(qty[k]);
    }
    printf("},\"requirements\":[");
    for (int k = 0; k < nr; k++) {
      printf("%s{\"key\":", k ? "," : "");
      put_str(reqs[k].key);
      printf(",\"op\":");
      put_str(reqs[k].op);
      printf(",\"values\":[");
      for (int v = 0; v < reqs[k].n_values; v++) {
        if (v) putchar(',');
        put_str(reqs[k].values[v]);
      }
      printf("]");
      if (reqs[k].has_gt) printf(",\"gt\":%lld", (long long)reqs[k].gt);
      if (reqs[k].has_lt) printf(",\"lt\":%lld", (long long)reqs[k].lt);
      printf("}");
    }
    printf("]}");
  }
  printf("],\"existingNodes\":[");
  int nn = ks_results_num_existing_nodes(r);
  for (int i = 0; i < nn; i++) {
    int idx = -1, np = 0;
    const int32_t* pods = NULL;
    if ((rc = ks_results_existing_node(r, i, &idx, &pods, &np)) != KS_OK) return fail("ks_results_existing_node", rc);
    printf("%s{\"stateNode\":%d,\"pods\":[", i ? "," : "", idx);
    for (int k = 0; k < np; k++) printf("%s%d", k ? "," : "", pods[k]);
    printf("]}");
  }
  printf("],\"podErrors\":{");
  int ne = ks_results_num_pod_errors(r);
  for (int i = 0; i < ne; i++) {
    int pod = -1;
    const char* msg = NULL;
    if ((rc = ks_results_pod_error(r, i, &pod, &msg)) != KS_OK) return fail("ks_results_pod_error", rc);
    printf("%s\"%d\":", i ? "," : "", pod);
    put_str(msg);
  }
  printf("},\"kernelMs\":%.6f}\n", ks_results_kernel_ms(r));
  /* out-of-range accessors are argument errors, not crashes */
  if (ks_results_nodeclaim(r, nc, NULL, NULL, NULL, NULL, NULL) != KS_ERR_ARG) return fail("range check", 0);
  ks_results_free(r);
  ks_problem_free(pb);
  free(snap);
  return 0;
}
