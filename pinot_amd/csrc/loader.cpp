// loader.cpp -- segment directory loader: pins an immutable Pinot segment straight from its on-disk directory
// (SURVEY.md 8(f) rank 4), without a Java-side copy.
//
//   V3 (the default format, SegmentGeneratorConfig.java:105; files under <dir>/v3/, SegmentDirectoryPaths.java:52):
//     metadata.properties, index_map (`<col>.<indexId>.startOffset|size`, column names may hold dots:
//     parsed from the right, ColumnIndexUtils.java:33-45) and columns.psf, whose entries are an 8-byte magic
//     0xdeadbeefdeafbead followed by the payload; `size` counts the magic (SingleFileIndexDirectory.java:72,
//     170-204, 213-305).
//   V1 (older segments): one file per index, <col>.dict, <col>.sv.unsorted.fwd / <col>.sv.sorted.fwd,
//     <col>.sv.raw.fwd (no-dictionary columns), <col>.bitmap.inv (V1Constants.java Indexes / Dict).
//
// metadata.properties keys (V1Constants.MetadataKeys, SegmentColumnarIndexCreator.addColumnMetadataInfo
// :519-541): segment.name, segment.total.docs, column.<col>.{cardinality, dataType, bitsPerElement,
// lengthOfEachEntry, isSorted, hasDictionary, isSingleValues}.  The files are memory-mapped and handed to the
// regular pin (ph_segment_pin copies them into HBM), so the bytes go from the page cache to the device once.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "ph_internal.h"

namespace ph {

namespace {

// java.util.Properties subset: `key = value` / `key: value` lines, '#' / '!' comments, backslash escapes
std::map<std::string, std::string> read_properties(const std::string& path) {
  std::ifstream in(path);
  if (!in) fail(PH_ERR_INVALID_ARGUMENT, "cannot open " + path);
  std::map<std::string, std::string> kv;
  std::string line;
  auto unescape = [&path](const std::string& s) {
    std::string o;
    for (size_t i = 0; i < s.size(); ++i) {
      if (s[i] == '\\' && i + 1 < s.size()) {
        const char c = s[++i];
        if (c == 't') o += '\t';
        else if (c == 'n') o += '\n';
        else if (c == 'u' && i + 4 < s.size()) {
          unsigned v = 0;
          bool hex = true;
          for (size_t k = i + 1; k <= i + 4; ++k) {
            const char h = s[k];
            const int d = (h >= '0' && h <= '9') ? h - '0' : (h >= 'a' && h <= 'f') ? h - 'a' + 10
                          : (h >= 'A' && h <= 'F') ? h - 'A' + 10 : -1;
            if (d < 0) hex = false;
            v = (v << 4) | (unsigned)(d < 0 ? 0 : d);
          }
          if (!hex) fail(PH_ERR_INVALID_ARGUMENT, "malformed \\uxxxx escape in " + path);
          i += 4;
          if (v < 0x80) o += (char)v;
          else o += '?';
        } else o += c;
      } else {
        o += s[i];
      }
    }
    return o;
  };
  auto trim = [](std::string s) {
    size_t a = s.find_first_not_of(" \t\r\f"), b = s.find_last_not_of(" \t\r\f");
    return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
  };
  while (std::getline(in, line)) {
    std::string t = trim(line);
    if (t.empty() || t[0] == '#' || t[0] == '!') continue;
    size_t sep = std::string::npos;
    for (size_t i = 0; i < t.size(); ++i) {
      if (t[i] == '\\') {
        ++i;
        continue;
      }
      if (t[i] == '=' || t[i] == ':') {
        sep = i;
        break;
      }
    }
    if (sep == std::string::npos) continue;
    // a repeated key is a list (commons-configuration: startree.v2.<i>.split.order, .function.column.pairs)
    const std::string key = unescape(trim(t.substr(0, sep))), val = unescape(trim(t.substr(sep + 1)));
    auto it = kv.find(key);
    if (it == kv.end()) kv[key] = val;
    else it->second += "," + val;
  }
  return kv;
}

// a whole decimal integer in [lo, hi] (metadata / index_map values are untrusted bytes)
int64_t to_i64(const std::string& s, const std::string& what, int64_t lo = INT64_MIN, int64_t hi = INT64_MAX) {
  size_t used = 0;
  long long v = 0;
  try {
    v = std::stoll(s, &used);
  } catch (...) {
    used = 0;
  }
  if (used == 0 || used != s.size() || v < lo || v > hi) fail(PH_ERR_INVALID_ARGUMENT, "bad " + what + ": '" + s + "'");
  return (int64_t)v;
}

struct Mapped {
  void* p = nullptr;
  size_t n = 0;
  Mapped() = default;
  Mapped(const Mapped&) = delete;
  Mapped& operator=(const Mapped&) = delete;
  ~Mapped() {
    if (p && n) munmap(p, n);
  }
};

std::unique_ptr<Mapped> map_file(const std::string& path, bool required) {
  const int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) {
    if (required) fail(PH_ERR_INVALID_ARGUMENT, "cannot open " + path);
    return nullptr;
  }
  struct stat st{};
  fstat(fd, &st);
  auto m = std::make_unique<Mapped>();
  m->n = (size_t)st.st_size;
  if (m->n) {
    m->p = mmap(nullptr, m->n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m->p == MAP_FAILED) {
      close(fd);
      m->p = nullptr;
      fail(PH_ERR_INVALID_ARGUMENT, "cannot map " + path);
    }
  }
  close(fd);
  return m;
}

bool file_exists(const std::string& p) {
  struct stat st{};
  return stat(p.c_str(), &st) == 0;
}

}  // namespace

// index_map of a V3 segment (SingleFileIndexDirectory.loadMap :213-247): `<col>.<indexId>.startOffset|size`
// properties; the key is split from the right because a column name may contain dots
// (ColumnIndexUtils.parseIndexMapKeys :33-45, whose Preconditions reject a key without both separators)
IndexMap read_index_map(const std::string& path) {
  IndexMap imap;
  auto im = read_properties(path);
  for (auto& kv : im) {
    const std::string& k = kv.first;
    const size_t a = k.rfind('.');
    if (a == std::string::npos) fail(PH_ERR_INVALID_ARGUMENT, "index_map: key separator not found: " + k);
    const size_t b = a == 0 ? std::string::npos : k.rfind('.', a - 1);
    if (b == std::string::npos) fail(PH_ERR_INVALID_ARGUMENT, "index_map: index separator not found: " + k);
    const std::string col = k.substr(0, b), idx = k.substr(b + 1, a - b - 1), what = k.substr(a + 1);
    auto& e = imap[{col, idx}];
    const int64_t v = to_i64(kv.second, "index_map value of " + k);
    if (what == "startOffset") e.first = v;
    else if (what == "size") e.second = v;
  }
  return imap;
}

namespace {

int32_t data_type_of(const std::string& t, const std::string& col) {
  // stored types (FieldSpec.DataType.getStoredType): BOOLEAN -> INT, TIMESTAMP -> LONG
  if (t == "INT" || t == "BOOLEAN") return PH_INT;
  if (t == "LONG" || t == "TIMESTAMP") return PH_LONG;
  if (t == "FLOAT") return PH_FLOAT;
  if (t == "DOUBLE") return PH_DOUBLE;
  if (t == "STRING") return PH_STRING;
  fail(PH_ERR_UNSUPPORTED, "column " + col + ": data type " + t + " is not on the GPU path");
}

}  // namespace

// the segment's doc count from its metadata.properties (0 if unreadable: the load itself reports the error), so a
// multi-device context places concurrent directory loads by their rows before any of them has pinned
int64_t segment_dir_num_docs(const char* dir_c) {
  if (!dir_c) return 0;
  try {
    std::string dir = dir_c;
    if (file_exists(dir + "/v3/metadata.properties")) dir += "/v3";
    auto meta = read_properties(dir + "/metadata.properties");
    auto it = meta.find("segment.total.docs");
    return it == meta.end() ? 0 : to_i64(it->second, "segment.total.docs", 0, INT32_MAX);
  } catch (const Error&) {
    return 0;
  }
}

void star_tree_add_impl(ph_segment* seg, const ph_star_tree_desc* d);  // startree.cpp

ph_segment* segment_load_dir_impl(Context* ctx, const char* dir_c, const char* const* want, int32_t nwant) {
  if (!dir_c) fail(PH_ERR_INVALID_ARGUMENT, "null segment directory");
  std::string dir = dir_c;
  const bool v3 = file_exists(dir + "/v3/metadata.properties") || file_exists(dir + "/index_map");
  if (file_exists(dir + "/v3/metadata.properties")) dir += "/v3";
  auto meta = read_properties(dir + "/metadata.properties");
  auto get = [&](const std::string& k) -> const std::string* {
    auto it = meta.find(k);
    return it == meta.end() ? nullptr : &it->second;
  };
  const std::string* docs_s = get("segment.total.docs");
  if (!docs_s) fail(PH_ERR_INVALID_ARGUMENT, "metadata.properties without segment.total.docs");
  const std::string seg_name = get("segment.name") ? *get("segment.name") : dir;
  const int64_t num_docs = to_i64(*docs_s, "segment.total.docs", 0, INT32_MAX);
  // only zero padding loads (ColumnMetadataImpl.java:297-300: unescapeJava(segment.padding.character) must be
  // "\0"; a missing key -- pre-2016 '%'-padded segments -- fails the load)
  {
    const std::string* pad = get("segment.padding.character");
    if (!pad || !((pad->size() == 1 && (*pad)[0] == '\0') || *pad == "\\u0000"))
      fail(PH_ERR_INVALID_ARGUMENT, "Got non-zero string padding: " + (pad ? *pad : std::string("(none)")));
  }

  // columns: the names behind column.<col>.cardinality (a column name may contain dots; the property is the
  // last component)
  std::vector<std::string> all;
  for (auto& kv : meta) {
    const std::string& k = kv.first;
    const std::string suffix = ".cardinality";
    if (k.rfind("column.", 0) == 0 && k.size() > 7 + suffix.size() &&
        k.compare(k.size() - suffix.size(), suffix.size(), suffix) == 0)
      all.push_back(k.substr(7, k.size() - 7 - suffix.size()));
  }
  std::vector<std::string> cols;
  const bool explicit_cols = want && nwant > 0;
  if (explicit_cols) {
    std::set<std::string> have(all.begin(), all.end());
    for (int32_t i = 0; i < nwant; ++i) {
      if (!want[i] || !have.count(want[i])) fail(PH_ERR_INVALID_ARGUMENT, std::string("column not in segment: ") + (want[i] ? want[i] : "(null)"));
      cols.push_back(want[i]);
    }
  } else {
    cols = all;
  }

  // index_map (V3): <col>.<indexId>.<startOffset|size>, split from the right
  IndexMap imap;  // (col, index) -> (start, size)
  std::unique_ptr<Mapped> psf;
  if (v3) {
    imap = read_index_map(dir + "/index_map");
    psf = map_file(dir + "/columns.psf", true);
  }
  std::vector<std::unique_ptr<Mapped>> v1files;
  // V3 buffer of (col, index): the payload after the 8-byte magic (SingleFileIndexDirectory.java:197-204)
  auto v3_buffer = [&](const std::string& col, const std::string& idx, const void** ptr, uint64_t* size) {
    auto it = imap.find({col, idx});
    if (it == imap.end()) return false;
    const int64_t start = it->second.first, sz = it->second.second;
    if (start < 0 || sz < 8 || (uint64_t)start > psf->n || (uint64_t)sz > psf->n - (uint64_t)start)
      fail(PH_ERR_INVALID_ARGUMENT, "index_map entry out of columns.psf: " + col + "." + idx);
    const uint8_t* base = static_cast<const uint8_t*>(psf->p) + start;
    uint64_t magic = 0;
    for (int i = 0; i < 8; ++i) magic = (magic << 8) | base[i];
    if (magic != 0xdeadbeefdeafbeadull) fail(PH_ERR_INVALID_ARGUMENT, "bad magic in columns.psf for " + col + "." + idx);
    *ptr = base + 8;
    *size = (uint64_t)(sz - 8);
    return true;
  };
  auto v1_buffer = [&](const std::string& file, bool required, const void** ptr, uint64_t* size) {
    auto m = map_file(dir + "/" + file, required);
    if (!m) return false;
    *ptr = m->p;
    *size = m->n;
    v1files.push_back(std::move(m));
    return true;
  };

  std::vector<ph_column_desc> descs;
  for (auto& c : cols) {
    auto prop = [&](const char* p) { return get("column." + c + "." + p); };
    const std::string* sv = prop("isSingleValues");
    const std::string* hd = prop("hasDictionary");
    const bool single = !sv || *sv == "true";
    const bool dict = !hd || *hd == "true";
    const std::string* dt = prop("dataType");
    if (!dt) fail(PH_ERR_INVALID_ARGUMENT, "column " + c + " without dataType");
    const bool fixed_raw = !dict && *dt != "STRING" && *dt != "BYTES" && *dt != "JSON" && *dt != "BIG_DECIMAL";
    if (!single || (!dict && !fixed_raw)) {
      if (explicit_cols)
        fail(PH_ERR_UNSUPPORTED, "column " + c + ": only single-value dictionary or fixed-width raw columns are on the GPU path");
      continue;  // stays with the CPU plan (multi-value / variable-width raw columns)
    }
    ph_column_desc d{};
    d.name = c.c_str();
    d.data_type = data_type_of(*dt, c);
    if (!dict) {
      // raw forward index (ForwardIndexReaderFactory.createRawIndexReader): V3 index "forward_index", V1
      // <col>.sv.raw.fwd (V1Constants.Indexes.RAW_SV_FORWARD_INDEX_FILE_EXTENSION)
      d.raw_forward_index = 1;
      const bool ok = v3 ? v3_buffer(c, "forward_index", &d.forward_index, &d.forward_index_size)
                         : v1_buffer(c + ".sv.raw.fwd", false, &d.forward_index, &d.forward_index_size);
      if (!ok) fail(PH_ERR_INVALID_ARGUMENT, "column " + c + ": raw forward index missing");
      if (v3) v3_buffer(c, "range_index", &d.range_index, &d.range_index_size);
      else v1_buffer(c + ".bitmap.range", false, &d.range_index, &d.range_index_size);
      descs.push_back(d);
      continue;
    }
    auto iprop = [&](const char* p, int64_t lo, int64_t hi) -> int32_t {
      const std::string* v = prop(p);
      if (!v) fail(PH_ERR_INVALID_ARGUMENT, "column " + c + " without " + p);
      return (int32_t)to_i64(*v, "column." + c + "." + p, lo, hi);
    };
    d.cardinality = iprop("cardinality", 0, INT32_MAX);
    d.bits_per_element = prop("bitsPerElement") ? iprop("bitsPerElement", 0, 32) : 0;
    d.is_sorted = prop("isSorted") && *prop("isSorted") == "true";
    d.dictionary_entry_size = d.data_type == PH_STRING ? iprop("lengthOfEachEntry", 0, INT32_MAX)
                                                       : ((d.data_type == PH_LONG || d.data_type == PH_DOUBLE) ? 8 : 4);
    bool ok_fwd, ok_dict;
    if (v3) {
      ok_fwd = v3_buffer(c, "forward_index", &d.forward_index, &d.forward_index_size);
      ok_dict = v3_buffer(c, "dictionary", &d.dictionary, &d.dictionary_size);
      v3_buffer(c, "inverted_index", &d.inverted_index, &d.inverted_index_size);
      v3_buffer(c, "range_index", &d.range_index, &d.range_index_size);  // StandardIndexes.RANGE_ID
    } else {
      ok_fwd = v1_buffer(c + (d.is_sorted ? ".sv.sorted.fwd" : ".sv.unsorted.fwd"), false, &d.forward_index,
                         &d.forward_index_size);
      ok_dict = v1_buffer(c + ".dict", false, &d.dictionary, &d.dictionary_size);
      v1_buffer(c + ".bitmap.inv", false, &d.inverted_index, &d.inverted_index_size);
      v1_buffer(c + ".bitmap.range", false, &d.range_index, &d.range_index_size);  // BITMAP_RANGE_INDEX_FILE_EXTENSION
    }
    if (!ok_fwd || !ok_dict) fail(PH_ERR_INVALID_ARGUMENT, "column " + c + ": forward index or dictionary missing");
    descs.push_back(d);
  }
  ph_segment_desc sd{};
  sd.name = seg_name.c_str();
  sd.num_docs = (int32_t)num_docs;
  sd.num_columns = (int32_t)descs.size();
  sd.columns = descs.data();
  ph_segment* seg = segment_pin_impl(ctx, &sd);  // copies the mapped bytes into HBM; the mappings close on return
  // star-trees (StarTreeLoaderUtils.loadStarTreeV2, StarTreeIndexContainer): star_tree_index holds every tree's
  // buffers, star_tree_index_map names them "<i>.<column>.<STAR_TREE | FORWARD_INDEX>.<OFFSET | SIZE>" (column "null"
  // for the tree itself), metadata.properties describes tree i under startree.v2.<i>.*.  A tree whose dimensions are
  // not all pinned (an explicit column list) cannot serve a query and is skipped.
  try {
    if (file_exists(dir + "/star_tree_index_map") && get("startree.v2.count")) {
      const int64_t ntrees = to_i64(*get("startree.v2.count"), "startree.v2.count", 0, 64);
      auto smap = read_properties(dir + "/star_tree_index_map");
      auto blob = map_file(dir + "/star_tree_index", true);
      auto list = [&](const std::string& k) {
        std::vector<std::string> out;
        const std::string* v = get(k);
        if (!v) fail(PH_ERR_INVALID_ARGUMENT, "metadata.properties without " + k);
        size_t a = 0;
        while (a <= v->size()) {
          size_t b = v->find(',', a);
          if (b == std::string::npos) b = v->size();
          std::string x = v->substr(a, b - a);
          while (!x.empty() && x.front() == ' ') x.erase(0, 1);
          while (!x.empty() && x.back() == ' ') x.pop_back();
          if (!x.empty()) out.push_back(x);
          a = b + 1;
        }
        return out;
      };
      auto buffer = [&](int64_t i, const std::string& col, const char* type, const void** ptr, uint64_t* size) {
        const std::string k = std::to_string(i) + "." + col + "." + type;
        auto o = smap.find(k + ".OFFSET"), n = smap.find(k + ".SIZE");
        if (o == smap.end() || n == smap.end()) fail(PH_ERR_INVALID_ARGUMENT, "star_tree_index_map without " + k);
        const int64_t off = to_i64(o->second, k, 0, INT64_MAX), sz = to_i64(n->second, k, 0, INT64_MAX);
        if ((uint64_t)off > blob->n || (uint64_t)sz > blob->n - (uint64_t)off)
          fail(PH_ERR_INVALID_ARGUMENT, "star_tree_index_map entry out of star_tree_index: " + k);
        *ptr = static_cast<const uint8_t*>(blob->p) + off;
        *size = (uint64_t)sz;
      };
      for (int64_t i = 0; i < ntrees; ++i) {
        const std::string pre = "startree.v2." + std::to_string(i) + ".";
        const std::vector<std::string> dims = list(pre + "split.order"), pairs = list(pre + "function.column.pairs");
        bool pinned = true;
        for (auto& d : dims) pinned = pinned && seg->columns.count(d) > 0;
        if (!pinned) continue;
        ph_star_tree_desc t{};
        buffer(i, "null", "STAR_TREE", &t.tree, &t.tree_size);
        t.num_docs = (int32_t)to_i64(get(pre + "total.docs") ? *get(pre + "total.docs") : std::string(),
                                     pre + "total.docs", 0, INT32_MAX);
        std::vector<const char*> dn, pn;
        std::vector<const void*> dp, pp;
        std::vector<uint64_t> ds, ps;
        for (auto& d : dims) {
          const void* ptr = nullptr;
          uint64_t size = 0;
          buffer(i, d, "FORWARD_INDEX", &ptr, &size);
          dn.push_back(d.c_str());
          dp.push_back(ptr);
          ds.push_back(size);
        }
        for (auto& pr : pairs) {
          const void* ptr = nullptr;
          uint64_t size = 0;
          const std::string k = std::to_string(i) + "." + pr + ".FORWARD_INDEX.OFFSET";
          if (smap.count(k)) buffer(i, pr, "FORWARD_INDEX", &ptr, &size);
          pn.push_back(pr.c_str());
          pp.push_back(ptr);
          ps.push_back(size);
        }
        t.num_dimensions = (int32_t)dims.size();
        t.dimensions = dn.data();
        t.dimension_forward_index = dp.data();
        t.dimension_forward_index_size = ds.data();
        t.num_metrics = (int32_t)pairs.size();
        t.metrics = pn.data();
        t.metric_forward_index = pp.data();
        t.metric_forward_index_size = ps.data();
        star_tree_add_impl(seg, &t);
      }
    }
  } catch (...) {
    ctx->pinned_rows -= seg->num_docs;
    delete seg;
    throw;
  }
  return seg;
}

}  // namespace ph
