// fuzz_host.cpp -- CPU sanitizer harness (SURVEY.md §5 race detection / sanitizers): the host
// parsers of libpinot_hip.so that read untrusted on-disk bytes, built with -fsanitize=address,undefined and fed
// every seed of a corpus plus seeded corruptions of it.  Test infrastructure only (tests/test_sanitize_cpu.py).
//
//   raw <file> <dataType> <numDocs>   raw_forward_index_decode   (rawfwd.cpp: chunk header, LZ4, Snappy)
//   inv <file> <cardinality>          build_bitmap_directory     (roaring.cpp: offsets + portable roaring)
//   dir <segment directory>           segment_load_dir_impl      (loader.cpp: metadata.properties, index_map,
//                                                                 columns.psf magic, V1 files)
//   map <index_map file>              read_index_map             (loader.cpp)
//
// Every call must either succeed or throw ph::Error (the C-ABI's status codes); a sanitizer report aborts the
// process (-fno-sanitize-recover=all).  Segment directories are copied to a scratch directory per mutation.
#include <sys/stat.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "ph_internal.h"

namespace ph {
[[noreturn]] void fail(int code, const std::string& msg) { throw Error{code, msg}; }
DeviceBuffer::~DeviceBuffer() {}
void DeviceBuffer::alloc(size_t, int) { fail(PH_ERR_DEVICE, "no device in the sanitizer harness"); }
// the loader's hand-off: every byte of every buffer it found must be readable (an out-of-map range would fault here)
ph_segment* segment_pin_impl(Context*, const ph_segment_desc* d) {
  volatile uint8_t acc = 0;
  for (int32_t i = 0; i < d->num_columns; ++i) {
    const ph_column_desc& c = d->columns[i];
    const void* p[3] = {c.forward_index, c.dictionary, c.inverted_index};
    const uint64_t n[3] = {c.forward_index_size, c.dictionary_size, c.inverted_index_size};
    for (int k = 0; k < 3; ++k)
      for (uint64_t j = 0; p[k] && j < n[k]; ++j) acc = acc ^ static_cast<const uint8_t*>(p[k])[j];
  }
  (void)acc;
  fail(PH_ERR_DEVICE, "harness: pin reached");
}
// (the pin never returns here, so the loader's star-tree step is not reached; these satisfy the link)
void star_tree_add_impl(ph_segment*, const ph_star_tree_desc*) { fail(PH_ERR_DEVICE, "harness: star-tree reached"); }
StarTree::~StarTree() {}
}  // namespace ph
ph_segment::~ph_segment() = default;

namespace {

std::vector<uint8_t> read_file(const std::string& p) {
  std::ifstream in(p, std::ios::binary);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
}

void write_file(const std::string& p, const std::vector<uint8_t>& b) {
  std::ofstream out(p, std::ios::binary | std::ios::trunc);
  out.write(reinterpret_cast<const char*>(b.data()), (std::streamsize)b.size());
}

// seeded corruptions: truncation, byte flips, 32-bit fields overwritten with extreme values, a zeroed span
std::vector<uint8_t> mutate(const std::vector<uint8_t>& src, std::mt19937_64& rng) {
  std::vector<uint8_t> b = src;
  const int kind = (int)(rng() % 4);
  if (b.empty()) return b;
  if (kind == 0) {
    b.resize(rng() % b.size());
  } else if (kind == 1) {
    const int flips = 1 + (int)(rng() % 8);
    for (int i = 0; i < flips; ++i) b[rng() % b.size()] ^= (uint8_t)(1u << (rng() % 8));
  } else if (kind == 2) {
    static const uint32_t ext[] = {0u, 0xffffffffu, 0x7fffffffu, 0x80000000u, 0x10000u, 0xffffu};
    const int n = 1 + (int)(rng() % 4);
    for (int i = 0; i < n && b.size() >= 4; ++i) {
      const size_t at = (rng() % (b.size() - 3)) & ~(size_t)3;
      const uint32_t v = (rng() % 2) ? ext[rng() % 6] : (uint32_t)rng();
      memcpy(&b[at], &v, 4);
    }
  } else {
    const size_t at = rng() % b.size(), len = std::min<size_t>(b.size() - at, 1 + rng() % 64);
    memset(&b[at], 0, len);
  }
  return b;
}

struct Tally {
  long ok = 0, rejected = 0;
};

template <class F>
void run_one(F&& f, Tally& t) {
  try {
    f();
    ++t.ok;
  } catch (const ph::Error&) {
    ++t.rejected;
  }
}

int32_t dtype_of(const std::string& s) {
  if (s == "INT") return PH_INT;
  if (s == "LONG") return PH_LONG;
  if (s == "FLOAT") return PH_FLOAT;
  if (s == "DOUBLE") return PH_DOUBLE;
  return PH_STRING;
}

void copy_tree(const std::string& from, const std::string& to) {
  const std::string cmd = "rm -rf '" + to + "' && cp -r '" + from + "' '" + to + "'";
  if (system(cmd.c_str()) != 0) {
    fprintf(stderr, "copy failed: %s\n", cmd.c_str());
    exit(2);
  }
}

std::vector<std::string> list_files(const std::string& dir) {
  std::vector<std::string> out;
  const std::string cmd = "find '" + dir + "' -type f";
  FILE* p = popen(cmd.c_str(), "r");
  char line[4096];
  while (p && fgets(line, sizeof line, p)) {
    std::string s(line);
    while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
    out.push_back(s);
  }
  if (p) pclose(p);
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: fuzz_host <manifest> <scratch dir> <mutations per seed> [seed]\n");
    return 2;
  }
  const std::string manifest = argv[1], scratch = argv[2];
  const int per_seed = atoi(argv[3]);
  std::mt19937_64 rng(argc > 4 ? strtoull(argv[4], nullptr, 10) : 20261017ull);
  std::ifstream mf(manifest);
  std::string line;
  Tally seeds, muts;
  while (std::getline(mf, line)) {
    std::istringstream ls(line);
    std::string kind, path;
    ls >> kind >> path;
    if (kind == "raw") {
      std::string dt;
      int64_t n = 0;
      ls >> dt >> n;
      const auto src = read_file(path);
      std::vector<int64_t> out((size_t)std::max<int64_t>(1, n));
      auto call = [&](const std::vector<uint8_t>& b) {
        ph::raw_forward_index_decode(b.data(), b.size(), dtype_of(dt), n, out.data());
      };
      Tally one;
      run_one([&] { call(src); }, one);
      if (one.ok != 1) {
        fprintf(stderr, "valid seed rejected: %s\n", line.c_str());
        return 3;
      }
      ++seeds.ok;
      for (int i = 0; i < per_seed; ++i) {
        const auto b = mutate(src, rng);
        run_one([&] { call(b); }, muts);
      }
    } else if (kind == "inv") {
      int32_t card = 0;
      ls >> card;
      const auto src = read_file(path);
      auto call = [&](const std::vector<uint8_t>& b) {
        ph::Column c;
        c.cardinality = card;
        c.inverted = b;
        if (!c.inverted.empty()) ph::build_bitmap_directory(c);
      };
      Tally one;
      run_one([&] { call(src); }, one);
      if (one.ok != 1) {
        fprintf(stderr, "valid seed rejected: %s\n", line.c_str());
        return 3;
      }
      ++seeds.ok;
      for (int i = 0; i < per_seed; ++i) {
        const auto b = mutate(src, rng);
        run_one([&] { call(b); }, muts);
      }
    } else if (kind == "map") {
      const auto src = read_file(path);
      const std::string tmp = scratch + "/index_map.fuzz";
      Tally one;
      run_one([&] { (void)ph::read_index_map(path); }, one);
      if (one.ok != 1) {
        fprintf(stderr, "valid seed rejected: %s\n", line.c_str());
        return 3;
      }
      ++seeds.ok;
      for (int i = 0; i < per_seed; ++i) {
        write_file(tmp, mutate(src, rng));
        run_one([&] { (void)ph::read_index_map(tmp); }, muts);
      }
    } else if (kind == "dir") {
      // the valid directory reaches the (stubbed) pin: PH_ERR_DEVICE "pin reached" counts as accepted
      auto load = [&](const std::string& d) {
        try {
          (void)ph::segment_load_dir_impl(nullptr, d.c_str(), nullptr, 0);
        } catch (const ph::Error& e) {
          if (e.code == PH_ERR_DEVICE && e.msg == "harness: pin reached") return;
          throw;
        }
      };
      Tally one;
      run_one([&] { load(path); }, one);
      if (one.ok != 1) {
        fprintf(stderr, "valid seed rejected: %s\n", line.c_str());
        return 3;
      }
      ++seeds.ok;
      const std::vector<std::string> files = list_files(path);
      const std::string work = scratch + "/dir.fuzz";
      for (int i = 0; i < per_seed && !files.empty(); ++i) {
        copy_tree(path, work);
        const std::string f = files[rng() % files.size()];
        const std::string rel = f.substr(path.size());
        write_file(work + rel, mutate(read_file(f), rng));
        run_one([&] { load(work); }, muts);
      }
    } else if (!kind.empty() && kind[0] != '#') {
      fprintf(stderr, "unknown manifest line: %s\n", line.c_str());
      return 2;
    }
  }
  printf("seeds accepted %ld; mutations: %ld accepted, %ld rejected with a status code; no sanitizer report\n",
         seeds.ok, muts.ok, muts.rejected);
  return 0;
}
