// TFRecord (+GZIP) writer/reader for flat scalar-feature tf.train.Example
// records — the on-disk format of the reference's TF pipeline
// (tensorflow2/data.py:108-131 writes it, :171-210 reads it) without
// TensorFlow: the Example protobuf is encoded/decoded by hand and CRC32C is
// computed with a slicing-by-8 table. C ABI, loaded from Python via ctypes.
//
// Record framing: u64 len | u32 masked_crc32c(len) | bytes | u32 masked_crc32c(bytes).
// Example := { 1: Features { 1: repeated MapEntry { 1: key, 2: Feature } } }
// Feature := oneof { 1: BytesList, 2: FloatList{1: packed float},
//                    3: Int64List{1: packed varint} }
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

uint32_t g_crc_tab[8][256];
bool g_crc_init = false;

void crc_init() {
  if (g_crc_init) return;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    g_crc_tab[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t)
      g_crc_tab[t][i] = (g_crc_tab[t - 1][i] >> 8) ^ g_crc_tab[0][g_crc_tab[t - 1][i] & 255];
  g_crc_init = true;
}

uint32_t crc32c(const uint8_t* p, size_t n) {
  crc_init();
  uint32_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    w ^= c;
    c = g_crc_tab[7][w & 255] ^ g_crc_tab[6][(w >> 8) & 255] ^ g_crc_tab[5][(w >> 16) & 255] ^
        g_crc_tab[4][(w >> 24) & 255] ^ g_crc_tab[3][(w >> 32) & 255] ^
        g_crc_tab[2][(w >> 40) & 255] ^ g_crc_tab[1][(w >> 48) & 255] ^ g_crc_tab[0][w >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) c = g_crc_tab[0][(c ^ *p++) & 255] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

uint32_t masked(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xA282EAD8u; }

void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}

bool get_varint(const uint8_t*& p, const uint8_t* e, uint64_t& v) {
  v = 0;
  for (int sh = 0; sh < 64 && p < e; sh += 7) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7F) << sh;
    if (!(b & 0x80)) return true;
  }
  return false;
}

void put_ld(std::string& s, int field, const std::string& body) {
  put_varint(s, ((uint64_t)field << 3) | 2);
  put_varint(s, body.size());
  s += body;
}

// One sink abstraction over FILE* / gzFile.
struct Sink {
  FILE* f = nullptr;
  gzFile g = nullptr;
  bool write(const void* p, size_t n) {
    if (g) return gzwrite(g, p, (unsigned)n) == (int)n;
    return fwrite(p, 1, n, f) == n;
  }
};

struct Source {
  FILE* f = nullptr;
  gzFile g = nullptr;
  bool read(void* p, size_t n) {
    if (g) return gzread(g, p, (unsigned)n) == (int)n;
    return fread(p, 1, n, f) == n;
  }
  void close() {
    if (g) gzclose(g);
    if (f) fclose(f);
  }
};

bool open_src(Source& s, const char* path, int gz) {
  if (gz) s.g = gzopen(path, "rb");
  else s.f = fopen(path, "rb");
  return s.g || s.f;
}

// Decode one Example into columns. types: 0 = int64, 1 = float32.
// Returns number of matched features, -1 on a malformed record.
int decode_example(const uint8_t* p, const uint8_t* e,
                   const std::unordered_map<std::string, int>& col, const int* types,
                   void** outs, int64_t row) {
  int matched = 0;
  uint64_t tag, len;
  while (p < e) {  // Example
    if (!get_varint(p, e, tag)) return -1;
    if ((tag & 7) != 2 || !get_varint(p, e, len) || len > (uint64_t)(e - p)) return -1;
    const uint8_t* fe = p + len;
    if ((tag >> 3) != 1) { p = fe; continue; }
    while (p < fe) {  // Features: map entries
      if (!get_varint(p, fe, tag) || (tag & 7) != 2 || !get_varint(p, fe, len) ||
          len > (uint64_t)(fe - p))
        return -1;
      const uint8_t* me = p + len;
      std::string key;
      const uint8_t* fv = nullptr;
      const uint8_t* fv_end = nullptr;
      while (p < me) {
        uint64_t t2, l2;
        if (!get_varint(p, me, t2) || (t2 & 7) != 2 || !get_varint(p, me, l2) ||
            l2 > (uint64_t)(me - p))
          return -1;
        if ((t2 >> 3) == 1) key.assign((const char*)p, l2);
        else if ((t2 >> 3) == 2) { fv = p; fv_end = p + l2; }
        p += l2;
      }
      auto it = col.find(key);
      if (it != col.end() && fv) {
        const int c = it->second;
        // Feature: oneof kind
        const uint8_t* q = fv;
        uint64_t kt, kl;
        if (!get_varint(q, fv_end, kt) || (kt & 7) != 2 || !get_varint(q, fv_end, kl)) return -1;
        const uint8_t* le = q + kl;
        const int kind = (int)(kt >> 3);
        // List: field 1, packed (wt 2) or unpacked (wt 0 / 5); take the first value
        uint64_t vt;
        if (!get_varint(q, le, vt)) return -1;
        double val = 0;
        bool have = false;
        if ((vt & 7) == 2) {
          uint64_t pl;
          if (!get_varint(q, le, pl) || pl == 0) return -1;
          if (kind == 3) { uint64_t v; if (!get_varint(q, le, v)) return -1; val = (double)(int64_t)v; have = true;
            if (types[c] == 0) { ((int64_t*)outs[c])[row] = (int64_t)v; ++matched; continue; } }
          else if (kind == 2) { float f; memcpy(&f, q, 4); val = f; have = true; }
        } else if ((vt & 7) == 0 && kind == 3) {
          uint64_t v; if (!get_varint(q, le, v)) return -1;
          if (types[c] == 0) { ((int64_t*)outs[c])[row] = (int64_t)v; ++matched; continue; }
          val = (double)(int64_t)v; have = true;
        } else if ((vt & 7) == 5 && kind == 2) {
          float f; memcpy(&f, q, 4); val = f; have = true;
        }
        if (!have) return -1;
        if (types[c] == 0) ((int64_t*)outs[c])[row] = (int64_t)val;
        else ((float*)outs[c])[row] = (float)val;
        ++matched;
      }
    }
  }
  return matched;
}

}  // namespace

extern "C" {

uint32_t tdfo_crc32c(const uint8_t* p, size_t n) { return crc32c(p, n); }
uint32_t tdfo_masked_crc32c(const uint8_t* p, size_t n) { return masked(crc32c(p, n)); }

// Write nrows Examples with ncols scalar features. types: 0 int64 (values
// given as int64 arrays), 1 float32. Returns 0 on success.
int tdfo_tfrecord_write(const char* path, int gz, int ncols, const char** names, const int* types,
                        const void** cols, int64_t nrows) {
  Sink s;
  if (gz) s.g = gzopen(path, "wb6");
  else s.f = fopen(path, "wb");
  if (!s.g && !s.f) return -1;
  std::string feats, entry, feat, lst, ex;
  for (int64_t r = 0; r < nrows; ++r) {
    feats.clear();
    for (int c = 0; c < ncols; ++c) {
      lst.clear();
      std::string packed;
      if (types[c] == 0) {
        put_varint(packed, (uint64_t)((const int64_t*)cols[c])[r]);
      } else {
        const float f = ((const float*)cols[c])[r];
        packed.append((const char*)&f, 4);
      }
      put_ld(lst, 1, packed);
      feat.clear();
      put_ld(feat, types[c] == 0 ? 3 : 2, lst);
      entry.clear();
      put_ld(entry, 1, std::string(names[c]));
      put_ld(entry, 2, feat);
      put_ld(feats, 1, entry);
    }
    ex.clear();
    put_ld(ex, 1, feats);
    const uint64_t len = ex.size();
    const uint32_t lc = masked(crc32c((const uint8_t*)&len, 8));
    const uint32_t dc = masked(crc32c((const uint8_t*)ex.data(), ex.size()));
    if (!s.write(&len, 8) || !s.write(&lc, 4) || !s.write(ex.data(), ex.size()) ||
        !s.write(&dc, 4)) {
      if (s.g) gzclose(s.g); else fclose(s.f);
      return -2;
    }
  }
  if (s.g) gzclose(s.g); else fclose(s.f);
  return 0;
}

// Count records (verifying CRCs when check_crc). Returns -1 on error.
int64_t tdfo_tfrecord_count(const char* path, int gz, int check_crc) {
  Source s;
  if (!open_src(s, path, gz)) return -1;
  int64_t n = 0;
  std::vector<uint8_t> buf;
  while (true) {
    uint64_t len;
    uint32_t lc, dc;
    if (!s.read(&len, 8)) break;
    if (!s.read(&lc, 4) || (check_crc && lc != masked(crc32c((const uint8_t*)&len, 8)))) { n = -1; break; }
    buf.resize(len);
    if (!s.read(buf.data(), len) || !s.read(&dc, 4)) { n = -1; break; }
    if (check_crc && dc != masked(crc32c(buf.data(), len))) { n = -1; break; }
    ++n;
  }
  s.close();
  return n;
}

// Read up to max_rows records into column buffers; returns rows read or a
// negative error (-2 corrupt record, -3 missing feature).
int64_t tdfo_tfrecord_read(const char* path, int gz, int ncols, const char** names,
                           const int* types, void** outs, int64_t max_rows, int check_crc) {
  Source s;
  if (!open_src(s, path, gz)) return -1;
  std::unordered_map<std::string, int> col;
  for (int c = 0; c < ncols; ++c) col[names[c]] = c;
  std::vector<uint8_t> buf;
  int64_t r = 0;
  while (r < max_rows) {
    uint64_t len;
    uint32_t lc, dc;
    if (!s.read(&len, 8)) break;
    if (!s.read(&lc, 4)) { r = -2; break; }
    buf.resize(len);
    if (!s.read(buf.data(), len) || !s.read(&dc, 4)) { r = -2; break; }
    if (check_crc && (lc != masked(crc32c((const uint8_t*)&len, 8)) ||
                      dc != masked(crc32c(buf.data(), len)))) { r = -2; break; }
    const int m = decode_example(buf.data(), buf.data() + len, col, types, outs, r);
    if (m < 0) { r = -2; break; }
    if (m < ncols) { r = -3; break; }
    ++r;
  }
  s.close();
  return r;
}

}  // extern "C"
