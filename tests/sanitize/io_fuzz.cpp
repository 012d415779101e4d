// Host sanitizer driver for libkdfm_io (csrc/audio_io.cpp), built by tests/test_io_sanitize.py with
// -fsanitize=address,undefined -fno-sanitize-recover=all and linked against the library SOURCE (not
// the shipped .so), so every out-of-bounds read, overflow or UB in the FLAC/WAV parsers aborts.
//
// usage: io_fuzz <mutations-per-file> <seed> <scratch-dir> <file>...
//   1. every file: probe, whole decode, an offset/length window, and a too-small buffer (must be
//      rejected with KDFM_IO_ERR_ARG, never written past);
//   2. every file: <mutations> corrupted copies (bit flips, byte stomps, truncations, header
//      length fields set to extremes) decoded again: any status is fine, a crash or a sanitizer
//      report is not;
//   3. one multi-threaded collate of all files (threads = 4) into padded rows.
// Exit status 0 = no sanitizer report (the sanitizers abort the process otherwise).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kdfm_io.h"

namespace {

std::vector<uint8_t> read_file(const char* p) {
  std::vector<uint8_t> b;
  FILE* f = std::fopen(p, "rb");
  if (!f) return b;
  uint8_t buf[65536];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
  std::fclose(f);
  return b;
}

bool write_file(const std::string& p, const std::vector<uint8_t>& b) {
  FILE* f = std::fopen(p.c_str(), "wb");
  if (!f) return false;
  bool ok = std::fwrite(b.data(), 1, b.size(), f) == b.size();
  std::fclose(f);
  return ok;
}

struct Rng {  // xorshift64*: reproducible mutations from the seed on the command line
  uint64_t s;
  uint64_t next() {
    s ^= s >> 12;
    s ^= s << 25;
    s ^= s >> 27;
    return s * 2685821657736338717ULL;
  }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

// Decode a file fully; returns the status.  Buffers are sized from probe (clamped) so a lying
// header cannot make the driver itself allocate absurdly.
int decode_all(const char* path, int64_t* frames_out) {
  int32_t sr = 0, ch = 0, bits = 0;
  int64_t frames = 0;
  int rc = kdfm_audio_probe(path, &sr, &ch, &bits, &frames);
  if (rc != KDFM_IO_OK) return rc;
  if (frames < 0 || frames > (int64_t)1 << 24) frames = (int64_t)1 << 16;
  std::vector<float> out((size_t)frames + 1);
  int64_t n = 0;
  rc = kdfm_audio_decode(path, 0, -1, out.data(), (int64_t)out.size(), &n, &sr);
  if (rc == KDFM_IO_OK && (n < 0 || n > (int64_t)out.size())) {
    std::fprintf(stderr, "decode reported %lld samples for a %zu-float buffer\n", (long long)n, out.size());
    std::abort();
  }
  if (frames_out) *frames_out = n;
  return rc;
}

void mutate(std::vector<uint8_t>& b, Rng& r) {
  if (b.empty()) return;
  switch (r.below(5)) {
    case 0: {  // a few bit flips
      int k = 1 + (int)r.below(8);
      for (int i = 0; i < k; ++i) b[r.below(b.size())] ^= (uint8_t)(1u << r.below(8));
      break;
    }
    case 1: {  // stomp a run of bytes with 0x00 / 0xFF / random
      size_t at = r.below(b.size()), len = 1 + r.below(16);
      uint8_t v = (uint8_t)(r.below(3) == 0 ? 0x00 : r.below(2) ? 0xFF : r.next());
      for (size_t i = at; i < b.size() && i < at + len; ++i) b[i] = v;
      break;
    }
    case 2:  // truncation anywhere (including inside the header)
      b.resize(r.below(b.size()));
      break;
    case 3: {  // the header region, where lengths / sizes / counts live
      size_t lim = b.size() < 64 ? b.size() : 64;
      int k = 1 + (int)r.below(4);
      for (int i = 0; i < k; ++i) b[r.below(lim)] = (uint8_t)r.next();
      break;
    }
    default: {  // 32-bit little-endian field forced to an extreme
      if (b.size() < 8) break;
      size_t at = r.below(b.size() - 4);
      uint32_t v = r.below(2) ? 0xFFFFFFFFu : 0x7FFFFFFFu;
      std::memcpy(&b[at], &v, 4);
      break;
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s <mutations> <seed> <scratch-dir> <file>...\n", argv[0]);
    return 2;
  }
  const int muts = std::atoi(argv[1]);
  Rng rng{(uint64_t)std::strtoull(argv[2], nullptr, 10) * 0x9E3779B97F4A7C15ULL + 1};
  const std::string dir = argv[3];
  std::vector<const char*> files(argv + 4, argv + argc);
  long decoded = 0, rejected = 0;

  for (const char* p : files) {
    int64_t n = 0;
    int rc = decode_all(p, &n);
    if (rc != KDFM_IO_OK) {
      std::fprintf(stderr, "valid input %s failed: %s\n", p, kdfm_io_last_error());
      return 1;
    }
    // a window, then a buffer one float too small (must be refused, not overrun)
    std::vector<float> w(64);
    int64_t got = 0;
    int32_t sr = 0;
    rc = kdfm_audio_decode(p, n / 3, 64, w.data(), 64, &got, &sr);
    if (rc != KDFM_IO_OK || got > 64) {
      std::fprintf(stderr, "window decode of %s: rc %d, %lld samples\n", p, rc, (long long)got);
      return 1;
    }
    if (n > 1) {
      std::vector<float> small((size_t)n - 1);
      rc = kdfm_audio_decode(p, 0, -1, small.data(), n - 1, &got, &sr);
      if (rc != KDFM_IO_ERR_ARG) {
        std::fprintf(stderr, "short buffer for %s not refused (rc %d)\n", p, rc);
        return 1;
      }
    }
    // corrupted copies
    std::vector<uint8_t> orig = read_file(p);
    const char* ext = std::strrchr(p, '.');
    std::string q = dir + "/mut" + (ext ? ext : "");
    for (int m = 0; m < muts; ++m) {
      std::vector<uint8_t> b = orig;
      int rounds = 1 + (int)rng.below(3);
      for (int k = 0; k < rounds; ++k) mutate(b, rng);
      if (!write_file(q, b)) return 1;
      (decode_all(q.c_str(), nullptr) == KDFM_IO_OK ? decoded : rejected)++;
    }
  }

  // collate every valid file at once on 4 threads
  int64_t stride = 0;
  for (const char* p : files) {
    int32_t sr, ch, bits;
    int64_t fr = 0;
    if (kdfm_audio_probe(p, &sr, &ch, &bits, &fr) != KDFM_IO_OK) return 1;
    if (fr > stride) stride = fr;
  }
  std::vector<float> batch((size_t)stride * files.size(), -1.0f);
  std::vector<int64_t> lens(files.size());
  int rc = kdfm_audio_load_batch(files.data(), (int32_t)files.size(), nullptr, nullptr, batch.data(), stride,
                                 lens.data(), 0, 4);
  if (rc != KDFM_IO_OK) {
    std::fprintf(stderr, "collate failed: %s\n", kdfm_io_last_error());
    return 1;
  }
  for (size_t i = 0; i < files.size(); ++i)
    for (int64_t j = lens[i]; j < stride; ++j)
      if (batch[i * stride + j] != 0.0f) {
        std::fprintf(stderr, "row %zu not zero-padded at %lld\n", i, (long long)j);
        return 1;
      }
  std::printf("files %zu mutated-decoded %ld mutated-rejected %ld\n", files.size(), decoded, rejected);
  return 0;
}
