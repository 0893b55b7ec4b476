// Native batched WAV decode for the input pipeline (dataset.py:98-102: scipy.io.wavfile.read of
// one 16 kHz PCM16 clip per item, zero padded to 16000 samples).  The reference decodes one file
// per __getitem__ in the training process (DataLoader num_workers=0, training.py:77); here a
// batch of files is decoded by a small pool of host threads straight into a caller buffer
// (typically pinned, so the host-to-device copy that follows is one DMA).
//
// Supported: RIFF/WAVE, fmt tag 1 (PCM) or 0xFFFE (WAVE_FORMAT_EXTENSIBLE with the PCM
// sub-format), 16 bits per sample, one channel — the format of the speech-commands corpus.
// Chunks other than "fmt " and "data" are skipped (word-aligned, as RIFF requires).  A data chunk
// that claims more bytes than the file holds is read up to the end of the file.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/srk.h"

namespace {

constexpr int64_t kLen = 16000;

uint32_t rd32(const unsigned char* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
uint16_t rd16(const unsigned char* p) { return (uint16_t)(p[0] | p[1] << 8); }

// Returns the number of samples in the file (>= 0) or a negative SRK_WAV_ERR_* code; `out` is
// always fully written (the first 16000 samples, zero padded; all zero on error).
int64_t decode_one(const char* path, int16_t* out) {
  std::memset(out, 0, kLen * sizeof(int16_t));
  if (!path) return SRK_WAV_ERR_OPEN;
  FILE* f = std::fopen(path, "rb");
  if (!f) return SRK_WAV_ERR_OPEN;
  std::vector<unsigned char> buf;
  unsigned char tmp[65536];
  size_t got;
  while ((got = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
  const bool read_err = std::ferror(f) != 0;
  std::fclose(f);
  if (read_err) return SRK_WAV_ERR_OPEN;
  const size_t n = buf.size();
  const unsigned char* p = buf.data();
  if (n < 12 || std::memcmp(p, "RIFF", 4) != 0 || std::memcmp(p + 8, "WAVE", 4) != 0) return SRK_WAV_ERR_FORMAT;
  size_t pos = 12;
  bool have_fmt = false;
  while (pos + 8 <= n) {
    const unsigned char* ck = p + pos;
    const uint64_t size = rd32(ck + 4);
    const size_t body = pos + 8;
    if (std::memcmp(ck, "fmt ", 4) == 0) {
      if (size < 16 || body + 16 > n) return SRK_WAV_ERR_FORMAT;
      uint16_t tag = rd16(p + body);
      const uint16_t channels = rd16(p + body + 2), bits = rd16(p + body + 14);
      if (tag == 0xFFFE) {   // WAVE_FORMAT_EXTENSIBLE: sub-format GUID starts at byte 24 of the chunk
        if (size < 40 || body + 26 > n) return SRK_WAV_ERR_FORMAT;
        tag = rd16(p + body + 24);
      }
      if (tag != 1 || channels != 1 || bits != 16) return SRK_WAV_ERR_UNSUPPORTED;
      have_fmt = true;
    } else if (std::memcmp(ck, "data", 4) == 0) {
      if (!have_fmt) return SRK_WAV_ERR_FORMAT;
      const uint64_t avail = std::min<uint64_t>(size, n - body);
      const int64_t samples = (int64_t)(avail / 2);
      const int64_t copy = std::min<int64_t>(samples, kLen);
      for (int64_t i = 0; i < copy; ++i) out[i] = (int16_t)rd16(p + body + 2 * i);   // little-endian
      return samples;
    }
    pos = body + size + (size & 1);
  }
  return SRK_WAV_ERR_FORMAT;   // no data chunk
}

}  // namespace

extern "C" int srk_wav_read_batch(const char* const* paths, int64_t n, int16_t* out, int64_t* lengths, int n_threads) {
  if (n < 0 || (n > 0 && (!paths || !out || !lengths))) return SRK_ERR_INVALID;
  if (n == 0) return SRK_OK;
  int threads = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
  threads = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)threads, 16, n}));
  std::atomic<int64_t> next{0};
  auto work = [&]() {
    for (int64_t i; (i = next.fetch_add(1)) < n;)
      lengths[i] = decode_one(paths[i], out + i * kLen);
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) {
    try {
      pool.emplace_back(work);
    } catch (...) {
      break;   // fewer threads; the calling thread still drains the queue
    }
  }
  work();
  for (auto& t : pool) t.join();
  return SRK_OK;
}
