// npz_reader.cpp — the per-track feature files read on native threads (host only, no GPU).
//
// The reference reads every song's features with deepdish (`dd.io.load`,
// acoss/algorithms/algorithm_template.py:90; EarlyFusion.load_features,
// acoss/algorithms/earlyfusion_traile.py:88-99). This package reads the `.npz` twin of each file
// (acoss/features_io.py). np.load parses the zip directory and every member's .npy header in
// Python, so 15,000 files took 12-17 s on 16 threads: the GIL serialised them.
// Here a batch of files is indexed and read by a pool of std::threads inside ONE C call (ctypes
// releases the GIL for its duration), in two steps:
//   acoss_npz_index: per file, the zip central directory (zip64 extra fields included) and, per
//     member whose top-level key is requested, its .npy header (descr, fortran_order, shape) and
//     where its data starts (stored members: the file offset; deflated: the offset after inflating
//     the header);
//   acoss_npz_read: per member, its array bytes into a caller buffer (pread for stored members,
//     raw zlib inflate for deflated ones, as np.savez_compressed writes).
// The caller (features_io.load_many) allocates one numpy array per member between the two calls.
// Errors name the file; no exception crosses the ABI.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "acoss_hip.h"

namespace acoss {
void set_error(const char* fmt, ...);
void clear_error();
}  // namespace acoss

namespace {

struct File {
  int fd = -1;
  explicit File(const char* p) { fd = ::open(p, O_RDONLY | O_CLOEXEC); }
  ~File() {
    if (fd >= 0) ::close(fd);
  }
  bool read_at(void* dst, size_t n, int64_t off) const {
    char* d = static_cast<char*>(dst);
    while (n) {
      const ssize_t r = ::pread(fd, d, n, off);
      if (r <= 0) return false;
      d += r;
      n -= (size_t)r;
      off += r;
    }
    return true;
  }
  int64_t size() const {
    const off_t e = ::lseek(fd, 0, SEEK_END);
    return (int64_t)e;
  }
};

inline uint16_t u16(const unsigned char* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t u32(const unsigned char* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
inline uint64_t u64(const unsigned char* p) { return (uint64_t)u32(p) | ((uint64_t)u32(p + 4) << 32); }

struct Entry {
  std::string name;
  int method;
  int64_t comp, size, local_off;
};

// The zip central directory (end record, zip64 end record when present, zip64 extra fields).
bool central_directory(const File& f, std::vector<Entry>* out, std::string* err) {
  const int64_t fsz = f.size();
  if (fsz < 22) {
    *err = "not a zip file (too short)";
    return false;
  }
  const int64_t tail = std::min<int64_t>(fsz, 22 + 65535 + 20);
  std::vector<unsigned char> t((size_t)tail);
  if (!f.read_at(t.data(), (size_t)tail, fsz - tail)) {
    *err = "read error";
    return false;
  }
  int64_t eocd = -1;
  for (int64_t i = tail - 22; i >= 0; --i)
    if (u32(&t[(size_t)i]) == 0x06054b50u) {
      eocd = i;
      break;
    }
  if (eocd < 0) {
    *err = "no zip end-of-central-directory record";
    return false;
  }
  uint64_t n_ent = u16(&t[(size_t)eocd + 10]);
  uint64_t cd_size = u32(&t[(size_t)eocd + 12]);
  uint64_t cd_off = u32(&t[(size_t)eocd + 16]);
  if (eocd >= 20 && u32(&t[(size_t)eocd - 20]) == 0x07064b50u) {  // zip64 end locator
    const uint64_t z64 = u64(&t[(size_t)eocd - 20 + 8]);
    unsigned char r[56];
    if (!f.read_at(r, sizeof r, (int64_t)z64) || u32(r) != 0x06064b50u) {
      *err = "bad zip64 end record";
      return false;
    }
    n_ent = u64(r + 32);
    cd_size = u64(r + 40);
    cd_off = u64(r + 48);
  }
  if ((int64_t)(cd_off + cd_size) > fsz) {
    *err = "central directory past the end of the file";
    return false;
  }
  std::vector<unsigned char> cd((size_t)cd_size);
  if (!f.read_at(cd.data(), (size_t)cd_size, (int64_t)cd_off)) {
    *err = "read error (central directory)";
    return false;
  }
  size_t p = 0;
  for (uint64_t e = 0; e < n_ent; ++e) {
    if (p + 46 > cd.size() || u32(&cd[p]) != 0x02014b50u) {
      *err = "bad central directory entry";
      return false;
    }
    Entry en;
    en.method = u16(&cd[p + 10]);
    uint64_t comp = u32(&cd[p + 20]), size = u32(&cd[p + 24]), loff = u32(&cd[p + 42]);
    const int nl = u16(&cd[p + 28]), xl = u16(&cd[p + 30]), cl = u16(&cd[p + 32]);
    if (p + 46 + nl + xl + cl > cd.size()) {
      *err = "truncated central directory entry";
      return false;
    }
    en.name.assign(reinterpret_cast<const char*>(&cd[p + 46]), (size_t)nl);
    // zip64 extra (id 1): the 8-byte forms of the fields stored as 0xffffffff, in this order
    size_t x = p + 46 + nl;
    const size_t xe = x + xl;
    while (x + 4 <= xe) {
      const int id = u16(&cd[x]), sz = u16(&cd[x + 2]);
      if (id == 1) {
        size_t q = x + 4;
        if (size == 0xffffffffu && q + 8 <= x + 4 + sz) { size = u64(&cd[q]); q += 8; }
        if (comp == 0xffffffffu && q + 8 <= x + 4 + sz) { comp = u64(&cd[q]); q += 8; }
        if (loff == 0xffffffffu && q + 8 <= x + 4 + sz) { loff = u64(&cd[q]); q += 8; }
      }
      x += 4 + (size_t)sz;
    }
    en.comp = (int64_t)comp;
    en.size = (int64_t)size;
    en.local_off = (int64_t)loff;
    out->push_back(std::move(en));
    p += 46 + nl + xl + cl;
  }
  return true;
}

// The .npy header at the start of a member: descr, fortran_order, shape and the header length.
bool npy_header(const unsigned char* h, size_t n, acoss_npz_member* m, std::string* err) {
  if (n < 10 || std::memcmp(h, "\x93NUMPY", 6) != 0) {
    *err = "member is not a .npy array";
    return false;
  }
  const int major = h[6];
  size_t hl, hs;
  if (major == 1) {
    hl = u16(h + 8);
    hs = 10;
  } else {
    if (n < 12) {
      *err = "short .npy header";
      return false;
    }
    hl = u32(h + 8);
    hs = 12;
  }
  if (hs + hl > n) {
    *err = "short .npy header";
    return false;
  }
  const std::string d(reinterpret_cast<const char*>(h + hs), hl);
  auto value_after = [&](const char* key) -> size_t {
    const size_t k = d.find(key);
    if (k == std::string::npos) return std::string::npos;
    const size_t c = d.find(':', k);
    return c == std::string::npos ? c : d.find_first_not_of(' ', c + 1);
  };
  size_t v = value_after("'descr'");
  if (v == std::string::npos || (d[v] != '\'' && d[v] != '"')) {
    *err = "npy header without a plain descr (structured or object dtype)";
    return false;
  }
  const size_t ve = d.find(d[v], v + 1);
  if (ve == std::string::npos || ve - v - 1 >= sizeof(m->descr)) {
    *err = "bad npy descr";
    return false;
  }
  std::memset(m->descr, 0, sizeof(m->descr));
  std::memcpy(m->descr, d.data() + v + 1, ve - v - 1);
  if (std::strchr(m->descr, 'O')) {
    *err = "object arrays are not read (allow_pickle=False)";
    return false;
  }
  v = value_after("'fortran_order'");
  m->fortran = (v != std::string::npos && d.compare(v, 4, "True") == 0) ? 1 : 0;
  v = value_after("'shape'");
  if (v == std::string::npos || d[v] != '(') {
    *err = "bad npy shape";
    return false;
  }
  const size_t se = d.find(')', v);
  m->ndim = 0;
  size_t q = v + 1;
  while (q < se) {
    while (q < se && (d[q] == ' ' || d[q] == ',')) ++q;
    if (q >= se) break;
    if (m->ndim >= 8) {
      *err = "more than 8 dimensions";
      return false;
    }
    m->shape[m->ndim++] = std::strtoll(d.c_str() + q, nullptr, 10);
    while (q < se && d[q] != ',') ++q;
  }
  m->data_skip = (int64_t)(hs + hl);
  return true;
}

// Item size of a numpy descr: '<f4' -> 4, '|u1' -> 1, '<U6' -> 24 (UCS-4), '|S6' -> 6.
int64_t itemsize(const char* descr) {
  const char* p = descr;
  if (*p == '<' || *p == '>' || *p == '|' || *p == '=') ++p;
  const char kind = *p++;
  const long long n = std::strtoll(p, nullptr, 10);
  if (n <= 0) return -1;
  return kind == 'U' ? 4 * n : n;
}

// Inflate the first `want` bytes of a deflated member (raw deflate) starting at `off`.
bool inflate_prefix(const File& f, int64_t off, int64_t comp, unsigned char* dst, size_t want, std::string* err) {
  z_stream zs;
  std::memset(&zs, 0, sizeof zs);
  if (inflateInit2(&zs, -MAX_WBITS) != Z_OK) {
    *err = "zlib init failed";
    return false;
  }
  std::vector<unsigned char> in(1 << 16);
  int64_t done_in = 0;
  zs.next_out = dst;
  zs.avail_out = (uInt)want;
  int rc = Z_OK;
  while (zs.avail_out > 0 && rc != Z_STREAM_END) {
    if (zs.avail_in == 0) {
      const int64_t chunk = std::min<int64_t>((int64_t)in.size(), comp - done_in);
      if (chunk <= 0) break;
      if (!f.read_at(in.data(), (size_t)chunk, off + done_in)) {
        inflateEnd(&zs);
        *err = "read error (deflated member)";
        return false;
      }
      done_in += chunk;
      zs.next_in = in.data();
      zs.avail_in = (uInt)chunk;
    }
    rc = inflate(&zs, Z_NO_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) {
      inflateEnd(&zs);
      *err = "corrupt deflated member";
      return false;
    }
  }
  inflateEnd(&zs);
  if (zs.avail_out != 0) {
    *err = "deflated member shorter than its header says";
    return false;
  }
  return true;
}

bool wanted(const std::string& name, const std::vector<std::string>& keys) {
  if (keys.empty()) return true;
  const std::string top = name.substr(0, name.find('/'));
  return std::find(keys.begin(), keys.end(), top) != keys.end();
}

bool index_file(const char* path, const std::vector<std::string>& keys, int32_t fidx, std::vector<acoss_npz_member>* out,
                std::string* err) {
  File f(path);
  if (f.fd < 0) {
    *err = "cannot open";
    return false;
  }
  std::vector<Entry> ents;
  if (!central_directory(f, &ents, err)) return false;
  for (const Entry& e : ents) {
    if (e.name.size() < 4 || e.name.compare(e.name.size() - 4, 4, ".npy") != 0) continue;
    const std::string nm = e.name.substr(0, e.name.size() - 4);
    if (!wanted(nm, keys)) continue;
    if (e.method != 0 && e.method != 8) {
      *err = "member " + e.name + ": compression method " + std::to_string(e.method) + " (only stored / deflate)";
      return false;
    }
    unsigned char lh[30];
    if (!f.read_at(lh, 30, e.local_off) || u32(lh) != 0x04034b50u) {
      *err = "bad local header of " + e.name;
      return false;
    }
    acoss_npz_member m;
    std::memset(&m, 0, sizeof m);
    m.file = fidx;
    m.method = e.method;
    m.member_off = e.local_off + 30 + u16(lh + 26) + u16(lh + 28);
    m.comp_size = e.comp;
    m.npy_size = e.size;
    if (nm.size() >= sizeof(m.name)) {
      *err = "member name too long: " + nm;
      return false;
    }
    std::memcpy(m.name, nm.data(), nm.size());
    // the .npy header: at most 64 KiB + 12 bytes (format 1.0 caps it at 65535; 2.0 is rare)
    const size_t hmax = (size_t)std::min<int64_t>(e.size, 65536 + 12);
    std::vector<unsigned char> h(hmax);
    const bool ok = e.method == 0 ? f.read_at(h.data(), hmax, m.member_off)
                                  : inflate_prefix(f, m.member_off, e.comp, h.data(), hmax, err);
    if (!ok) {
      if (err->empty()) *err = "read error (member header)";
      return false;
    }
    if (!npy_header(h.data(), hmax, &m, err)) {
      *err = e.name + ": " + *err;
      return false;
    }
    const int64_t isz = itemsize(m.descr);
    if (isz <= 0) {
      *err = e.name + ": unsupported dtype " + m.descr;
      return false;
    }
    int64_t cnt = 1;
    for (int d = 0; d < m.ndim; ++d) cnt *= m.shape[d];
    m.nbytes = cnt * isz;
    if (m.data_skip + m.nbytes > m.npy_size) {
      *err = e.name + ": array data past the end of the member";
      return false;
    }
    out->push_back(m);
  }
  return true;
}

bool read_member(const File& f, const acoss_npz_member& m, void* dst, std::string* err) {
  if (m.nbytes == 0) return true;
  if (m.method == 0) {
    if (!f.read_at(dst, (size_t)m.nbytes, m.member_off + m.data_skip)) {
      *err = std::string("read error (") + m.name + ")";
      return false;
    }
    return true;
  }
  // deflated: inflate header + data, keep the data
  std::vector<unsigned char> all((size_t)(m.data_skip + m.nbytes));
  if (!inflate_prefix(f, m.member_off, m.comp_size, all.data(), all.size(), err)) return false;
  std::memcpy(dst, all.data() + m.data_skip, (size_t)m.nbytes);
  return true;
}

template <class F>
void parallel_for(int64_t n, int32_t n_threads, F fn) {
  int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
  nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n));
  std::atomic<int64_t> next(0);
  auto work = [&]() {
    for (int64_t i = next++; i < n; i = next++) fn(i);
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < nt; ++t) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
}

}  // namespace

extern "C" int acoss_npz_index(const char* const* paths, int32_t n_files, const char* keys, int32_t n_threads,
                               acoss_npz_member* out, int64_t max_out, int64_t* n_out) {
  acoss::clear_error();
  if (n_files < 0 || (n_files > 0 && !paths) || !n_out || max_out < 0 || (max_out > 0 && !out)) {
    acoss::set_error("acoss_npz_index: bad arguments");
    return ACOSS_E_ARG;
  }
  std::vector<std::string> kl;
  if (keys) {
    std::string s(keys);
    size_t p = 0;
    while (p <= s.size()) {
      const size_t e = s.find('\n', p);
      const std::string k = s.substr(p, e == std::string::npos ? std::string::npos : e - p);
      if (!k.empty()) kl.push_back(k);
      if (e == std::string::npos) break;
      p = e + 1;
    }
  }
  std::vector<std::vector<acoss_npz_member>> per((size_t)n_files);
  std::vector<std::string> errs((size_t)n_files);
  std::atomic<int> failed(-1);
  parallel_for(n_files, n_threads, [&](int64_t i) {
    if (failed.load() >= 0) return;
    if (!index_file(paths[i], kl, (int32_t)i, &per[(size_t)i], &errs[(size_t)i])) {
      int expect = -1;
      failed.compare_exchange_strong(expect, (int)i);
    }
  });
  if (failed.load() >= 0) {
    const int i = failed.load();
    acoss::set_error("%s: %s", paths[i], errs[(size_t)i].c_str());
    return ACOSS_E_ARG;
  }
  int64_t tot = 0;
  for (const auto& v : per) tot += (int64_t)v.size();
  *n_out = tot;
  if (tot > max_out) {
    acoss::set_error("acoss_npz_index: %lld members, room for %lld", (long long)tot, (long long)max_out);
    return ACOSS_E_ARG;
  }
  int64_t o = 0;
  for (const auto& v : per)
    for (const auto& m : v) out[o++] = m;
  return ACOSS_OK;
}

extern "C" int acoss_npz_read(const char* const* paths, const acoss_npz_member* members, int64_t n_members,
                              void* const* dst, int32_t n_threads) {
  acoss::clear_error();
  if (n_members < 0 || (n_members > 0 && (!paths || !members || !dst))) {
    acoss::set_error("acoss_npz_read: bad arguments");
    return ACOSS_E_ARG;
  }
  // members of one file are contiguous (acoss_npz_index's order): one task per file
  std::vector<int64_t> starts;
  for (int64_t i = 0; i < n_members; ++i)
    if (i == 0 || members[i].file != members[i - 1].file) starts.push_back(i);
  starts.push_back(n_members);
  const int64_t nf = (int64_t)starts.size() - 1;
  std::vector<std::string> errs((size_t)std::max<int64_t>(nf, 0));
  std::atomic<int64_t> failed(-1);
  parallel_for(nf, n_threads, [&](int64_t t) {
    if (failed.load() >= 0) return;
    const acoss_npz_member& m0 = members[starts[(size_t)t]];
    File f(paths[m0.file]);
    bool ok = f.fd >= 0;
    if (!ok) errs[(size_t)t] = "cannot open";
    for (int64_t i = starts[(size_t)t]; ok && i < starts[(size_t)t + 1]; ++i)
      ok = read_member(f, members[i], dst[i], &errs[(size_t)t]);
    if (!ok) {
      int64_t expect = -1;
      failed.compare_exchange_strong(expect, t);
    }
  });
  if (failed.load() >= 0) {
    const int64_t t = failed.load();
    acoss::set_error("%s: %s", paths[members[starts[(size_t)t]].file], errs[(size_t)t].c_str());
    return ACOSS_E_ARG;
  }
  return ACOSS_OK;
}
