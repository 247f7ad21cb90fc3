// bg_starch.hip — Starch v2 archives (BEDOPS' compressed BED) decoded on the host into the
// BED text the GPU loader parses ("Starch input decode (CPU, starchApi.hpp)").
//
// Reference: interfaces/general-headers/data/starch/starchApi.hpp (Starch::isStarch :645-676,
// the per-stream bzip2/gzip readers setupBzip2Works :1217 / setupGzipWorks :1281, the line
// loop extractLine :1490-1760), interfaces/src/data/starch/unstarchHelpers.c
// (UNSTARCH_sReverseTransformIgnoringHeaderedInput :884-1160, the token split
// UNSTARCH_createInverseTransformTokens :1538-1585), starchMetadataHelpers.h:104-109 (layout).
// Archive layout (v2.x): 4 magic bytes ca 5c ad e5, then one compressed stream per
// chromosome back to back, then the JSON metadata ("compressionFormat" 0 = bzip2, 1 = gzip;
// "streams": [{"chromosome", "size"}, ...] in archive order), then a 128-byte footer whose
// first 20 characters are the metadata's byte offset (decimal, zero-padded); the reader
// seeks to 127 bytes before the end (starchMetadataHelpers.c:1113). v1.x archives put the
// JSON first and the streams right after it (legacy: padded to 8192 bytes;
// starchMetadataHelpers.c:985-1060 finds the first compression magic behind it).
// Each stream is a transformed BED: "p<N>" sets the current length, "<delta>[\t<rest>]" is a
// row whose start is delta after the previous row's end (the first row of a stream: delta
// itself when it has a rest), end = start + length; track/browser/'#'/'@' lines are skipped
// (the C++ readers never print headers, starchApi.hpp:1515-1517). Streams decode in parallel
// host threads; the text is concatenated in archive order. bzip2 comes from the system
// libbz2 (dlopen; the image has the library but not its header), gzip from zlib.
#include <ctype.h>
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <cinttypes>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bedgpu.h"

namespace {

const unsigned char kMagic[4] = {0xca, 0x5c, 0xad, 0xe5};
const size_t kFooter = 127;         // STARCH2_MD_FOOTER_LENGTH - 1 bytes on disk
const size_t kHeader = 4;           // STARCH2_MD_HEADER_BYTE_LENGTH
const size_t kOffsetDigits = 20;    // STARCH2_MD_FOOTER_CUMULATIVE_RECORD_SIZE_LENGTH

// ------------------------------------------------------------------ minimal JSON reader
struct Json {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  double num = 0;
  std::string str;
  std::vector<Json> items;                             // ARR
  std::vector<std::pair<std::string, Json>> members;   // OBJ
  const Json* get(const char* k) const {
    for (const auto& m : members)
      if (m.first == k) return &m.second;
    return nullptr;
  }
};
struct JsonParser {
  const char* p;
  const char* e;
  bool ok = true;
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p; }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(e - p) >= n && !memcmp(p, s, n)) { p += n; return true; }
    return false;
  }
  std::string string() {
    std::string out;
    ++p;  // opening quote
    while (p < e && *p != '"') {
      if (*p == '\\' && p + 1 < e) {
        ++p;
        switch (*p) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'u': {  // \uXXXX (ASCII range only; chromosome names are ASCII)
            unsigned v = 0;
            for (int k = 0; k < 4 && p + 1 < e; ++k) {
              ++p;
              v = v * 16 + (unsigned)(isdigit((unsigned char)*p) ? *p - '0' : (tolower(*p) - 'a' + 10));
            }
            out += (char)(v & 0x7f);
            break;
          }
          default: out += *p;
        }
        ++p;
      } else {
        out += *p++;
      }
    }
    if (p >= e) ok = false;
    else ++p;
    return out;
  }
  Json value(int depth = 0) {
    Json v;
    ws();
    if (p >= e || depth > 32) { ok = false; return v; }
    if (*p == '{') {
      v.kind = Json::OBJ;
      ++p;
      ws();
      if (p < e && *p == '}') { ++p; return v; }
      while (ok) {
        ws();
        if (p >= e || *p != '"') { ok = false; break; }
        std::string k = string();
        ws();
        if (p >= e || *p != ':') { ok = false; break; }
        ++p;
        v.members.emplace_back(k, value(depth + 1));
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == '}') { ++p; break; }
        ok = false;
      }
    } else if (*p == '[') {
      v.kind = Json::ARR;
      ++p;
      ws();
      if (p < e && *p == ']') { ++p; return v; }
      while (ok) {
        v.items.push_back(value(depth + 1));
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == ']') { ++p; break; }
        ok = false;
      }
    } else if (*p == '"') {
      v.kind = Json::STR;
      v.str = string();
    } else if (lit("true")) {
      v.kind = Json::BOOL;
      v.num = 1;
    } else if (lit("false")) {
      v.kind = Json::BOOL;
    } else if (lit("null")) {
      v.kind = Json::NUL;
    } else {
      char* q = nullptr;
      v.kind = Json::NUM;
      v.num = strtod(std::string(p, (size_t)std::min<ptrdiff_t>(e - p, 64)).c_str(), &q);
      const char* s = p;
      while (p < e && (isdigit((unsigned char)*p) || *p == '-' || *p == '+' || *p == '.' || *p == 'e' || *p == 'E')) ++p;
      if (p == s) ok = false;
    }
    return v;
  }
};

// a size given as a JSON number or a decimal string ("size": "284")
bool as_u64(const Json* v, uint64_t& out) {
  if (!v) return false;
  if (v->kind == Json::NUM) { out = (uint64_t)v->num; return v->num >= 0; }
  if (v->kind == Json::STR && !v->str.empty()) {
    char* q = nullptr;
    out = strtoull(v->str.c_str(), &q, 10);
    return q && *q == '\0';
  }
  return false;
}

// ------------------------------------------------------------------ decompressors
// bzip2's public stream ABI (bzlib.h of libbz2 1.0.x)
struct bz_stream_abi {
  char* next_in;
  unsigned int avail_in;
  unsigned int total_in_lo32, total_in_hi32;
  char* next_out;
  unsigned int avail_out;
  unsigned int total_out_lo32, total_out_hi32;
  void* state;
  void* (*bzalloc)(void*, int, int);
  void (*bzfree)(void*, void*);
  void* opaque;
};
struct Bz2 {
  int (*init)(bz_stream_abi*, int, int) = nullptr;
  int (*dec)(bz_stream_abi*) = nullptr;
  int (*end)(bz_stream_abi*) = nullptr;
  bool load() {
    static void* h = nullptr;
    if (!h) h = dlopen("libbz2.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libbz2.so.1.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return false;
    init = (int (*)(bz_stream_abi*, int, int))dlsym(h, "BZ2_bzDecompressInit");
    dec = (int (*)(bz_stream_abi*))dlsym(h, "BZ2_bzDecompress");
    end = (int (*)(bz_stream_abi*))dlsym(h, "BZ2_bzDecompressEnd");
    return init && dec && end;
  }
};
enum { BZ_OK_ = 0, BZ_STREAM_END_ = 4 };

bool bunzip(const Bz2& bz, const unsigned char* in, size_t n, std::string& out) {
  size_t pos = 0;
  while (pos < n) {  // concatenated bzip2 members decode one after another
    bz_stream_abi s;
    memset(&s, 0, sizeof(s));
    if (bz.init(&s, 0, 0) != BZ_OK_) return false;
    s.next_in = (char*)(in + pos);
    s.avail_in = (unsigned)std::min<size_t>(n - pos, 1u << 30);
    int rc = BZ_OK_;
    do {
      const size_t o = out.size();
      out.resize(o + (1u << 20));
      s.next_out = &out[o];
      s.avail_out = 1u << 20;
      rc = bz.dec(&s);
      out.resize(o + (1u << 20) - s.avail_out);
      if (rc != BZ_OK_ && rc != BZ_STREAM_END_) { bz.end(&s); return false; }
      if (rc == BZ_OK_ && s.avail_in == 0 && s.avail_out != 0) { bz.end(&s); return false; }  // truncated
    } while (rc != BZ_STREAM_END_);
    const size_t used = (size_t)s.next_in - (size_t)(in + pos);
    bz.end(&s);
    if (used == 0) return false;
    pos += used;
  }
  return true;
}

bool inflate_all(const unsigned char* in, size_t n, std::string& out) {
  size_t pos = 0;
  while (pos < n) {
    z_stream z;
    memset(&z, 0, sizeof(z));
    if (inflateInit2(&z, 15 + 32) != Z_OK) return false;  // zlib or gzip wrapper
    z.next_in = (Bytef*)(in + pos);
    z.avail_in = (uInt)std::min<size_t>(n - pos, 1u << 30);
    int rc = Z_OK;
    do {
      const size_t o = out.size();
      out.resize(o + (1u << 20));
      z.next_out = (Bytef*)&out[o];
      z.avail_out = 1u << 20;
      rc = inflate(&z, Z_NO_FLUSH);
      out.resize(o + (1u << 20) - z.avail_out);
      if (rc != Z_OK && rc != Z_STREAM_END) { inflateEnd(&z); return false; }
      if (rc == Z_OK && z.avail_in == 0 && z.avail_out != 0) { inflateEnd(&z); return false; }
    } while (rc != Z_STREAM_END);
    const size_t used = (size_t)(z.next_in - (Bytef*)(in + pos));
    inflateEnd(&z);
    if (used == 0) return false;
    pos += used;
  }
  return true;
}

// ------------------------------------------------------------------ reverse transform
bool is_header(const char* s, size_t n) {
  auto pre = [&](const char* h) { size_t k = strlen(h); return n >= k && !memcmp(s, h, k); };
  return pre("track") || pre("browser") || pre("@") || pre("#");  // "##" is a '#' line too
}
// strtoull(tok, NULL, 10) on a token that is not NUL-terminated
uint64_t dec_u64(const char* s, size_t n) {
  char b[32];
  const size_t k = std::min<size_t>(n, sizeof(b) - 1);
  memcpy(b, s, k);
  b[k] = '\0';
  return strtoull(b, nullptr, 10);
}
void transform(const std::string& chrom, const std::string& raw, std::string& out) {
  int64_t start = 0, plen = 0, last_end = 0;
  char num[48];
  size_t i = 0;
  while (i < raw.size()) {
    size_t j = raw.find('\n', i);
    if (j == std::string::npos) j = raw.size();
    const char* ln = raw.data() + i;
    const size_t n = j - i;
    i = j + 1;
    if (n == 0 || is_header(ln, n)) continue;
    const char* tab = (const char*)memchr(ln, '\t', n);
    const size_t n1 = tab ? (size_t)(tab - ln) : n;
    const char* tok2 = tab ? tab + 1 : ln + n;
    const size_t n2 = tab ? n - n1 - 1 : 0;
    if (n2 > 0) {
      const int64_t d = (int64_t)dec_u64(ln, n1);
      start = last_end > 0 ? last_end + d : d;
      last_end = start + plen;
      out += chrom;
      snprintf(num, sizeof(num), "\t%" PRId64 "\t%" PRId64 "\t", start, last_end);
      out += num;
      out.append(tok2, n2);
      out += '\n';
    } else if (n1 > 0 && ln[0] == 'p') {
      plen = (int64_t)dec_u64(ln + 1, n1 - 1);
    } else {
      start = last_end + (int64_t)dec_u64(ln, n1);
      last_end = start + plen;
      out += chrom;
      snprintf(num, sizeof(num), "\t%" PRId64 "\t%" PRId64 "\n", start, last_end);
      out += num;
    }
  }
}

}  // namespace

static bool is_v2(const void* data, uint64_t n) {
  return data && n >= kHeader + kFooter && !memcmp(data, kMagic, 4);
}
// v1.x: the archive opens with its JSON metadata (hasStarchRevision1Header)
static bool is_v1(const void* data, uint64_t n) {
  if (!data || n < 16 || ((const char*)data)[0] != '{') return false;
  const size_t k = (size_t)std::min<uint64_t>(n, 512);
  const std::string head((const char*)data, k);
  return head.find("\"archive\"") != std::string::npos && head.find("\"starch\"") != std::string::npos;
}

extern "C" int bg_starch_is(const void* data, uint64_t n) { return is_v2(data, n) || is_v1(data, n); }

extern "C" int bg_starch_decode(const void* data, uint64_t n, const char* chrom, char** out,
                                uint64_t* outlen, char* err, uint64_t errcap) {
  auto fail = [&](int code, const std::string& m) {
    if (err && errcap) snprintf(err, (size_t)errcap, "%s", m.c_str());
    return code;
  };
  if (!data || !out || !outlen) return BG_E_ARG;
  *out = nullptr;
  *outlen = 0;
  if (!bg_starch_is(data, n)) return fail(BG_E_PARSE, "not a Starch archive");
  const unsigned char* d = (const unsigned char*)data;
  const bool v2 = is_v2(data, n);
  uint64_t mdoff = 0, data0 = kHeader, mdend = n;
  Json md;
  if (v2) {
    const char* foot = (const char*)d + n - kFooter;
    for (size_t k = 0; k < kOffsetDigits; ++k) {
      if (!isdigit((unsigned char)foot[k])) return fail(BG_E_PARSE, "Starch footer: bad metadata offset");
      mdoff = mdoff * 10 + (uint64_t)(foot[k] - '0');
    }
    if (mdoff < kHeader || mdoff > n - kFooter) return fail(BG_E_PARSE, "Starch footer: metadata offset out of range");
    mdend = mdoff;
    JsonParser P{(const char*)d + mdoff, foot};
    md = P.value();
    if (!P.ok || md.kind != Json::OBJ) return fail(BG_E_PARSE, "Starch metadata is not valid JSON");
  } else {
    JsonParser P{(const char*)d, (const char*)d + n};
    md = P.value();
    if (!P.ok || md.kind != Json::OBJ) return fail(BG_E_PARSE, "Starch metadata is not valid JSON");
    // the streams start at the first bzip2 / gzip / zlib magic behind the JSON
    uint64_t q = (uint64_t)(P.p - (const char*)d);
    const uint64_t lim = std::min<uint64_t>(n, std::max<uint64_t>(q + 64, 8192 + 64));
    while (q + 2 < lim && !((d[q] == 'B' && d[q + 1] == 'Z' && d[q + 2] == 'h') ||
                            (d[q] == 0x1f && d[q + 1] == 0x8b) || (d[q] == 0x78 && (d[q + 1] == 0x01 || d[q + 1] == 0x9c || d[q + 1] == 0xda))))
      ++q;
    data0 = q;
  }
  const Json* arch = md.get("archive");
  const Json* streams = md.get("streams");
  if (!arch || !streams || streams->kind != Json::ARR) return fail(BG_E_PARSE, "Starch metadata without archive/streams");
  const Json* ver = arch->get("version");
  const Json* major = ver ? ver->get("major") : nullptr;
  if (!major || major->kind != Json::NUM || major->num != (v2 ? 2 : 1))
    return fail(BG_E_UNSUPPORTED, "Starch archive version not read by this build");
  const Json* cf = arch->get("compressionFormat");
  const int comp = (cf && cf->kind == Json::NUM) ? (int)cf->num : 0;
  if (comp != 0 && comp != 1) return fail(BG_E_PARSE, "unknown Starch compression format");
  Bz2 bz;
  if (comp == 0 && !bz.load()) return fail(BG_E_UNSUPPORTED, "libbz2 is not available to read bzip2 Starch streams");
  struct Job {
    std::string chrom;
    uint64_t off = 0, size = 0;
    std::string text;
    bool ok = true;
  };
  std::vector<Job> jobs;
  uint64_t off = data0;
  for (const Json& s : streams->items) {
    Job j;
    const Json* c = s.get("chromosome");
    if (!c || c->kind != Json::STR || !as_u64(s.get("size"), j.size))
      return fail(BG_E_PARSE, "Starch stream record without chromosome/size");
    j.chrom = c->str;
    j.off = off;
    off += j.size;
    if (off > mdend) return fail(BG_E_PARSE, "Starch stream sizes run past the metadata");
    if (!chrom || j.chrom == chrom) jobs.push_back(std::move(j));
  }
  auto run = [&](Job& j) {
    std::string raw;
    j.ok = comp == 0 ? bunzip(bz, d + j.off, (size_t)j.size, raw) : inflate_all(d + j.off, (size_t)j.size, raw);
    if (j.ok) transform(j.chrom, raw, j.text);
  };
  const size_t nt = std::min<size_t>(jobs.size(), std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (size_t k = t; k < jobs.size(); k += nt) run(jobs[k]);
    });
  for (auto& x : th) x.join();
  uint64_t total = 0;
  for (const Job& j : jobs) {
    if (!j.ok) return fail(BG_E_PARSE, "Starch stream of " + j.chrom + " could not be decompressed");
    total += j.text.size();
  }
  char* buf = (char*)malloc(total + 1);
  if (!buf) return BG_E_NOMEM;
  uint64_t o = 0;
  for (const Job& j : jobs) {
    memcpy(buf + o, j.text.data(), j.text.size());
    o += j.text.size();
  }
  buf[o] = '\0';
  *out = buf;
  *outlen = o;
  return 0;
}
