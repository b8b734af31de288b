// mmap CSV reader + dictionary encoder + group-by → CSR transactions.
//
// Replaces the reference's polars (Rust) ingest path: `pl.read_csv` (machine-learning/main.py:153)
// and the group-bys at main.py:53-73, 87-95, 114-125, 169-171, 196-198.  Strings are
// dictionary-encoded to int32 codes in first-appearance order while the file is scanned once;
// every later group-by runs on integer codes (here or on the GPU), never on strings.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <deque>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "kmls/common.hpp"
#include "kmls/host.hpp"

namespace kmls {

namespace {

struct MappedFile {
  const char* data = nullptr;
  size_t size = 0;
  int fd = -1;
  explicit MappedFile(const std::string& path) {
    fd = ::open(path.c_str(), O_RDONLY);
    KMLS_CHECK(fd >= 0, "cannot open " + path);
    struct stat st;
    KMLS_CHECK(::fstat(fd, &st) == 0, "cannot stat " + path);
    size = (size_t)st.st_size;
    if (size) {
      void* p = ::mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      KMLS_CHECK(p != MAP_FAILED, "mmap failed for " + path);
      ::madvise(p, size, MADV_SEQUENTIAL);
      data = (const char*)p;
    }
  }
  ~MappedFile() {
    if (data) ::munmap((void*)data, size);
    if (fd >= 0) ::close(fd);
  }
};

// Dictionary with stable string storage; ids in first-appearance order.
struct Dict {
  std::deque<std::string> store;
  std::unordered_map<std::string_view, int32_t> map;
  int32_t get(std::string_view s) {
    auto it = map.find(s);
    if (it != map.end()) return it->second;
    store.emplace_back(s);
    int32_t id = (int32_t)map.size();
    map.emplace(std::string_view(store.back()), id);
    return id;
  }
};

// RFC-4180 field scanner.  Returns the position after the field's terminator (',' or EOL).
// `field` receives the unescaped value (`scratch` backs it when unescaping was needed).
inline size_t scan_field(const char* d, size_t pos, size_t end, std::string_view& field,
                         std::string& scratch, bool& eol) {
  eol = false;
  if (pos < end && d[pos] == '"') {
    size_t p = pos + 1;
    scratch.clear();
    bool simple = true;
    size_t start = p;
    while (p < end) {
      char c = d[p];
      if (c == '"') {
        if (p + 1 < end && d[p + 1] == '"') {  // escaped quote
          if (simple) { scratch.assign(d + start, p - start); simple = false; }
          scratch.push_back('"');
          p += 2;
          continue;
        }
        break;  // closing quote
      }
      if (!simple) scratch.push_back(c);
      ++p;
    }
    field = simple ? std::string_view(d + start, p - start) : std::string_view(scratch);
    p = std::min(p + 1, end);  // skip closing quote
    // move to terminator
    while (p < end && d[p] != ',' && d[p] != '\n' && d[p] != '\r') ++p;
    if (p >= end) { eol = true; return end; }
    if (d[p] == ',') return p + 1;
    eol = true;
    if (d[p] == '\r' && p + 1 < end && d[p + 1] == '\n') return p + 2;
    return p + 1;
  }
  size_t p = pos;
  while (p < end && d[p] != ',' && d[p] != '\n' && d[p] != '\r') ++p;
  field = std::string_view(d + pos, p - pos);
  if (p >= end) { eol = true; return end; }
  if (d[p] == ',') return p + 1;
  eol = true;
  if (d[p] == '\r' && p + 1 < end && d[p + 1] == '\n') return p + 2;
  return p + 1;
}

}  // namespace

EncodedTable read_csv_encoded(const std::string& path, const std::vector<std::string>& wanted) {
  MappedFile f(path);
  const char* d = f.data;
  const size_t end = f.size;
  EncodedTable out;
  size_t pos = 0;
  std::string scratch;
  std::string_view fld;
  bool eol = false;
  // header
  std::vector<std::string> header;
  while (pos < end) {
    pos = scan_field(d, pos, end, fld, scratch, eol);
    header.emplace_back(fld);
    if (eol) break;
  }
  KMLS_CHECK(!header.empty(), "empty csv " + path);
  // strip UTF-8 BOM
  if (header[0].size() >= 3 && (unsigned char)header[0][0] == 0xEF) header[0] = header[0].substr(3);
  std::vector<int> col_slot(header.size(), -1);
  for (size_t w = 0; w < wanted.size(); ++w) {
    auto it = std::find(header.begin(), header.end(), wanted[w]);
    KMLS_CHECK(it != header.end(), "column not found: " + wanted[w]);
    col_slot[it - header.begin()] = (int)w;
  }
  out.header = header;
  out.columns = wanted;
  std::vector<Dict> dicts(wanted.size());
  out.codes.assign(wanted.size(), {});
  const size_t approx_rows = end / 64 + 16;
  for (auto& c : out.codes) c.reserve(approx_rows);
  int64_t rows = 0;
  while (pos < end) {
    // skip blank lines
    if (d[pos] == '\n' || d[pos] == '\r') { ++pos; continue; }
    size_t col = 0;
    while (true) {
      pos = scan_field(d, pos, end, fld, scratch, eol);
      if (col < col_slot.size() && col_slot[col] >= 0) {
        int w = col_slot[col];
        out.codes[w].push_back(dicts[w].get(fld));
      }
      ++col;
      if (eol) break;
    }
    KMLS_CHECK(col == header.size(), "ragged csv row " + std::to_string(rows + 2) + " in " + path);
    ++rows;
  }
  out.n_rows = rows;
  out.uniques.resize(wanted.size());
  for (size_t w = 0; w < wanted.size(); ++w) {
    out.uniques[w].assign(dicts[w].store.begin(), dicts[w].store.end());
  }
  return out;
}

CSR group_to_csr(const int32_t* keys, const int32_t* vals, int64_t n, int32_t n_keys, bool dedup,
                 bool sort_rows) {
  CSR g;
  g.ptr.assign((size_t)n_keys + 1, 0);
  for (int64_t i = 0; i < n; ++i) g.ptr[(size_t)keys[i] + 1]++;
  for (int32_t k = 0; k < n_keys; ++k) g.ptr[k + 1] += g.ptr[k];
  g.idx.resize((size_t)n);
  std::vector<int64_t> fill(g.ptr.begin(), g.ptr.end() - 1);
  for (int64_t i = 0; i < n; ++i) g.idx[(size_t)fill[keys[i]]++] = vals[i];  // stable
  if (!dedup && !sort_rows) return g;
  std::vector<int64_t> nptr((size_t)n_keys + 1, 0);
  int64_t w = 0;
  for (int32_t k = 0; k < n_keys; ++k) {
    int32_t* b = g.idx.data() + g.ptr[k];
    int32_t* e = g.idx.data() + g.ptr[k + 1];
    if (sort_rows || dedup) std::sort(b, e);
    if (dedup) e = std::unique(b, e);
    nptr[k] = w;
    for (int32_t* p = b; p < e; ++p) g.idx[(size_t)w++] = *p;
  }
  nptr[n_keys] = w;
  g.idx.resize((size_t)w);
  g.ptr.swap(nptr);
  return g;
}

}  // namespace kmls
