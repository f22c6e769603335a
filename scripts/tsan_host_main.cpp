// ThreadSanitizer harness for the threaded host code of libkarpenter_amd (scripts/tsan_host.sh): the JSON
// parser's parallel array parse and the pod / NewTopology workers (ks_parallel.h) through the host-only
// entry points, and the snapshot reaper thread (ks_json.h release_async) through ks_cons_create, which
// releases the parsed document before it looks for a device (none here: that error is expected).
// Built with -fsanitize=thread against the TSan build of the host objects, so every access is instrumented
// (a TSan runtime preloaded into an uninstrumented Python interpreter deadlocks in CPython's own locks).
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

extern "C" int ks_problem_inspect(const char*, size_t, char**);
extern "C" int ks_cons_inspect(const char*, size_t, char**);
extern "C" int ks_cons_create(const char*, size_t, void**);
extern "C" const char* ks_last_error(void);
extern "C" void ks_free(void*);

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  std::ifstream f(argv[2]);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str(), mode = argv[1];
  char* out = nullptr;
  int rc;
  if (mode == "solve") {
    rc = ks_problem_inspect(s.data(), s.size(), &out);
  } else {
    rc = ks_cons_inspect(s.data(), s.size(), &out);
    if (rc == 0) {
      void* h = nullptr;
      const int rc2 = ks_cons_create(s.data(), s.size(), &h);  // parse + build + reaper; no device here
      printf("ks_cons_create without a device: %d (%s)\n", rc2, rc2 ? ks_last_error() : "ok");
    }
  }
  if (rc) {
    fprintf(stderr, "error %d: %s\n", rc, ks_last_error());
    return 1;
  }
  printf("%s: %.120s...\n", mode.c_str(), out);
  ks_free(out);
  return 0;
}
