// Development: host cost of the problem analysis behind okvisgpu_set_problems (runtime.cpp analyse())
// on one S50 window, CPU only (no HIP call is made). Unity build:
//   hipcc -std=c++17 -O3 -I include -I okvis2-x_amd/csrc scripts/analyse_bench.cpp \
//     okvis2-x_amd/csrc/synth.cpp -o /tmp/analyse_bench
#include "../okvis2-x_amd/csrc/runtime.cpp"

#include <chrono>
#include <cstdio>

int main(int argc, char** argv) {
  okvisgpu_synth_config cfg;
  okvisgpu_synth_default_config(&cfg, 50, 2000, 16000, 20251015);
  okvisgpu_synth_window* w = nullptr;
  if (okvisgpu_synth_create(&cfg, &w) != OKVISGPU_OK) return 1;
  std::vector<const okvisgpu_problem*> probs{okvisgpu_synth_problem(w)};
  std::map<std::tuple<int, int, int>, int> none;
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  double best = 1e30;
#ifdef OKG_ANALYSE_TIMING
  g_alast = std::chrono::steady_clock::now();
#endif
  for (int r = 0; r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    HostBatch B;
    analyse(probs, none, B);
    const auto t1 = std::chrono::steady_clock::now();
    best = std::min(best, std::chrono::duration<double, std::milli>(t1 - t0).count());
  }
  std::printf("analyse S50: best %.3f ms over %d reps\n", best, reps);
#ifdef OKG_ANALYSE_TIMING
  const char* names[11] = {"(between)", "params+const", "active/priors/f-blocks", "obs sort", "visits", "extr visits",
                           "groups/segments/parts", "imu/priors/ranges", "f-block lists", "pairs", "tiles/lists"};
  for (int i = 0; i < 11; ++i) std::printf("  %-24s %.3f ms/rep\n", names[i], g_atime[i] / reps);
#endif
  return 0;
}
