// Standalone stress test of the native clip reader core, built with host sanitizers by
// tests/test_native_sanitizers.py (-fsanitize=thread; -fsanitize=address,undefined).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../csrc/runtime/clip_reader_core.h"

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const int nfiles = 6, frames = 40, fb = 3 * 17 * 23, hdr = 128;
  std::vector<std::string> paths;
  for (int f = 0; f < nfiles; ++f) {
    const std::string p = dir + "/clip_" + std::to_string(f) + ".raw";
    FILE* fp = std::fopen(p.c_str(), "wb");
    if (!fp) return 2;
    std::vector<unsigned char> buf(hdr + (size_t)frames * fb);
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = (unsigned char)((i * 131 + f * 7) & 255);
    std::fwrite(buf.data(), 1, buf.size(), fp);
    std::fclose(fp);
    paths.push_back(p);
  }
  pva::ClipReader reader;
  std::mt19937 rng(0);
  for (int it = 0; it < 50; ++it) {
    const int nthreads = 1 + (int)(rng() % 8);
    const int njobs = 1 + (int)(rng() % 12);
    std::vector<pva::ReadJob> jobs;
    int64_t off = 0;
    for (int j = 0; j < njobs; ++j) {
      pva::ReadJob r{paths[rng() % nfiles], hdr, fb, {}, off};
      const int n = 1 + (int)(rng() % 16);
      for (int k = 0; k < n; ++k) r.idx.push_back(rng() % frames);
      off += (int64_t)n * fb;
      jobs.push_back(r);
    }
    std::vector<unsigned char> dst(off);
    const std::string err = reader.read(dst.data(), off, jobs, nthreads);
    if (!err.empty()) { std::fprintf(stderr, "error: %s\n", err.c_str()); return 1; }
    for (const auto& r : jobs) {
      const int f = std::atoi(r.path.substr(r.path.rfind('_') + 1).c_str());
      for (size_t k = 0; k < r.idx.size(); ++k)
        for (int b = 0; b < fb; b += 97) {
          const size_t src = hdr + (size_t)r.idx[k] * fb + b;
          if (dst[r.dst_offset + k * fb + b] != (unsigned char)((src * 131 + f * 7) & 255)) {
            std::fprintf(stderr, "mismatch\n");
            return 1;
          }
        }
    }
  }
  // overflow is reported, not written
  std::vector<unsigned char> small(10);
  pva::ReadJob big{paths[0], hdr, fb, {0}, 0};
  if (reader.read(small.data(), 10, {big}, 2).empty()) return 1;
  std::puts("clip_reader_test ok");
  return 0;
}
