// FLAC decoder (host, C-ABI) for load_audio: the reference decodes audio files by
// piping them through the ffmpeg CLI (whisper/audio.py:25-62), which this image does
// not have.  This restates the FLAC stream format (STREAMINFO + frames of CONSTANT /
// VERBATIM / FIXED / LPC subframes with Rice-coded residuals and the four channel
// decorrelation modes) directly; the decoded samples are bit-exact, checked against
// the MD5 of the unencoded audio that every FLAC stream carries in STREAMINFO
// (tests/test_audio_io.py).  Down-mixing / resampling happen in Python (audio.py).
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "whisper_hip.h"

namespace {

struct Bits {
  const uint8_t* p;
  int64_t n, pos = 0;  // pos in bits
  bool bad = false;
  Bits(const uint8_t* d, int64_t len) : p(d), n(len) {}
  uint32_t bit() {
    if ((pos >> 3) >= n) { bad = true; return 0; }
    const uint32_t b = (p[pos >> 3] >> (7 - (pos & 7))) & 1u;
    ++pos;
    return b;
  }
  uint64_t u(int k) {  // k <= 64, MSB first
    uint64_t v = 0;
    while (k > 0) {
      if ((pos & 7) == 0 && k >= 8 && (pos >> 3) < n) {
        v = (v << 8) | p[pos >> 3];
        pos += 8;
        k -= 8;
      } else {
        v = (v << 1) | bit();
        --k;
      }
    }
    return v;
  }
  int64_t s(int k) {  // two's complement, k bits
    if (k == 0) return 0;
    const uint64_t v = u(k);
    return (int64_t)(v << (64 - k)) >> (64 - k);
  }
  uint32_t unary() {  // zeros before the next 1
    uint32_t q = 0;
    while (!bad) {
      if ((pos & 7) == 0 && (pos >> 3) < n && p[pos >> 3] == 0) {
        q += 8;
        pos += 8;
        continue;
      }
      if (bit()) break;
      ++q;
    }
    return q;
  }
  void align() { pos = (pos + 7) & ~int64_t(7); }
};

struct StreamInfo {
  int rate = 0, channels = 0, bps = 0;
  int64_t total = 0;
  int64_t frames_at = 0;  // byte offset of the first frame
};

std::string g_flac_err;

int ferr(int rc, const std::string& m) {
  g_flac_err = m;
  return rc;
}

int parse_header(const uint8_t* d, int64_t n, StreamInfo* si) {
  if (n < 42 || memcmp(d, "fLaC", 4) != 0) return ferr(-1, "not a FLAC stream");
  int64_t i = 4;
  bool have_info = false;
  while (true) {
    if (i + 4 > n) return ferr(-2, "truncated metadata");
    const int last = d[i] >> 7, type = d[i] & 127;
    const int64_t len = ((int64_t)d[i + 1] << 16) | ((int64_t)d[i + 2] << 8) | d[i + 3];
    if (i + 4 + len > n) return ferr(-2, "truncated metadata block");
    if (type == 0) {
      Bits b(d + i + 4, len);
      b.u(16);  // min block size
      b.u(16);  // max block size
      b.u(24);  // min frame size
      b.u(24);  // max frame size
      si->rate = (int)b.u(20);
      si->channels = (int)b.u(3) + 1;
      si->bps = (int)b.u(5) + 1;
      si->total = (int64_t)b.u(36);
      have_info = true;
    }
    i += 4 + len;
    if (last) break;
  }
  if (!have_info) return ferr(-3, "no STREAMINFO block");
  si->frames_at = i;
  return 0;
}

// residual of a FIXED / LPC subframe (partitioned Rice, 4- or 5-bit parameters)
bool residual(Bits& b, int bs, int order, int32_t* out) {
  const int method = (int)b.u(2);
  if (method > 1) return false;
  const int pbits = method == 0 ? 4 : 5, esc = method == 0 ? 15 : 31;
  const int po = (int)b.u(4);
  const int parts = 1 << po;
  if ((bs >> po) < order) return false;
  int k = order;
  for (int pi = 0; pi < parts; ++pi) {
    const int cnt = (bs >> po) - (pi == 0 ? order : 0);
    const int rp = (int)b.u(pbits);
    if (rp == esc) {
      const int nb = (int)b.u(5);
      for (int j = 0; j < cnt; ++j) out[k++] = (int32_t)b.s(nb);
    } else {
      for (int j = 0; j < cnt; ++j) {
        const uint64_t q = b.unary();
        const uint64_t v = (q << rp) | (rp ? b.u(rp) : 0);
        out[k++] = (int32_t)((int64_t)(v >> 1) ^ -(int64_t)(v & 1));
      }
    }
    if (b.bad) return false;
  }
  return true;
}

bool subframe(Bits& b, int bs, int bps, int64_t* s, std::vector<int32_t>& res) {
  if (b.bit() != 0) return false;
  const int type = (int)b.u(6);
  int wasted = 0;
  if (b.bit()) wasted = (int)b.unary() + 1;
  bps -= wasted;
  if (bps <= 0) return false;
  if (type == 0) {
    const int64_t v = b.s(bps);
    for (int i = 0; i < bs; ++i) s[i] = v;
  } else if (type == 1) {
    for (int i = 0; i < bs; ++i) s[i] = b.s(bps);
  } else if (type >= 8 && type <= 12) {
    const int order = type - 8;
    for (int i = 0; i < order; ++i) s[i] = b.s(bps);
    res.resize(bs);
    if (!residual(b, bs, order, res.data())) return false;
    for (int i = order; i < bs; ++i) {
      int64_t p = 0;
      switch (order) {
        case 1: p = s[i - 1]; break;
        case 2: p = 2 * s[i - 1] - s[i - 2]; break;
        case 3: p = 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3]; break;
        case 4: p = 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]; break;
        default: break;
      }
      s[i] = p + res[i];
    }
  } else if (type >= 32) {
    const int order = type - 31;
    for (int i = 0; i < order; ++i) s[i] = b.s(bps);
    const int prec = (int)b.u(4) + 1;
    if (prec == 16) return false;
    const int shift = (int)b.s(5);
    if (shift < 0) return false;
    int64_t c[32];
    for (int j = 0; j < order; ++j) c[j] = b.s(prec);
    res.resize(bs);
    if (!residual(b, bs, order, res.data())) return false;
    for (int i = order; i < bs; ++i) {
      int64_t acc = 0;
      for (int j = 0; j < order; ++j) acc += c[j] * s[i - 1 - j];
      s[i] = res[i] + (acc >> shift);
    }
  } else {
    return false;
  }
  if (wasted)
    for (int i = 0; i < bs; ++i) s[i] = (int64_t)((uint64_t)s[i] << wasted);
  return !b.bad;
}

}  // namespace

extern "C" {

const char* wh_flac_last_error(void) { return g_flac_err.c_str(); }

int wh_flac_info(const uint8_t* data, int64_t n, int* sample_rate, int* channels, int* bits_per_sample,
                 int64_t* total_samples) {
  if (!data) return ferr(-1, "null data");
  StreamInfo si;
  const int rc = parse_header(data, n, &si);
  if (rc) return rc;
  if (sample_rate) *sample_rate = si.rate;
  if (channels) *channels = si.channels;
  if (bits_per_sample) *bits_per_sample = si.bps;
  if (total_samples) *total_samples = si.total;
  return 0;
}

int wh_flac_decode(const uint8_t* data, int64_t n, int32_t* out, int64_t cap_frames, int64_t* n_frames) {
  if (!data || !out || !n_frames) return ferr(-1, "null argument");
  StreamInfo si;
  int rc = parse_header(data, n, &si);
  if (rc) return rc;
  const int C = si.channels;
  Bits b(data, n);
  b.pos = si.frames_at * 8;
  int64_t done = 0;
  std::vector<int64_t> ch[8];
  std::vector<int32_t> res;
  while ((b.pos >> 3) + 2 < n) {
    if (b.u(14) != 0x3FFE) return ferr(-4, "lost frame sync at byte " + std::to_string(b.pos / 8 - 2));
    b.u(1);  // reserved
    b.u(1);  // blocking strategy
    const int bsc = (int)b.u(4), src = (int)b.u(4), chc = (int)b.u(4), ssc = (int)b.u(3);
    b.u(1);
    // frame / sample number, UTF-8-like: leading ones of the first byte = length
    const uint32_t f0 = (uint32_t)b.u(8);
    int extra = 0;
    for (uint32_t m = 0x80; m && (f0 & m); m >>= 1) ++extra;
    for (int k = 1; k < extra; ++k) b.u(8);
    int bs = 0;
    if (bsc == 1) bs = 192;
    else if (bsc >= 2 && bsc <= 5) bs = 576 << (bsc - 2);
    else if (bsc == 6) bs = (int)b.u(8) + 1;
    else if (bsc == 7) bs = (int)b.u(16) + 1;
    else if (bsc >= 8) bs = 256 << (bsc - 8);
    else return ferr(-5, "reserved block size");
    if (src == 12) b.u(8);
    else if (src == 13 || src == 14) b.u(16);
    else if (src == 15) return ferr(-5, "invalid sample rate code");
    static const int ssz[8] = {0, 8, 12, 0, 16, 20, 24, 32};
    const int bps = ssc == 0 ? si.bps : ssz[ssc];
    if (bps == 0) return ferr(-5, "reserved sample size");
    b.u(8);  // CRC-8 of the header
    const int nch = chc < 8 ? chc + 1 : 2;
    if (chc > 10 || nch != C) return ferr(-5, "channel assignment does not match STREAMINFO");
    for (int c = 0; c < nch; ++c) {
      ch[c].resize(bs);
      const bool side = (chc == 8 && c == 1) || (chc == 9 && c == 0) || (chc == 10 && c == 1);
      if (!subframe(b, bs, bps + (side ? 1 : 0), ch[c].data(), res))
        return ferr(-6, "bad subframe in frame at sample " + std::to_string(done));
    }
    b.align();
    b.u(16);  // CRC-16 of the frame
    if (b.bad) return ferr(-6, "truncated frame");
    for (int i = 0; i < bs; ++i) {
      int64_t v[8];
      for (int c = 0; c < nch; ++c) v[c] = ch[c][i];
      if (chc == 8) v[1] = v[0] - v[1];          // left / side
      else if (chc == 9) v[0] = v[0] + v[1];     // side / right
      else if (chc == 10) {                      // mid / side
        const int64_t mid = (v[0] * 2) | (v[1] & 1), sd = v[1];
        v[0] = (mid + sd) >> 1;
        v[1] = (mid - sd) >> 1;
      }
      if (done >= cap_frames) return ferr(-7, "output capacity exceeded");
      for (int c = 0; c < nch; ++c) out[done * C + c] = (int32_t)v[c];
      ++done;
    }
  }
  *n_frames = done;
  return 0;
}

}  // extern "C"
