#include "gguf.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

namespace fa {

static thread_local std::string g_gguf_err;
const char* gguf_error() { return g_gguf_err.c_str(); }

float half_to_float_host(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000) << 16;
  uint32_t exp = (h >> 10) & 0x1F, man = h & 0x3FF, bits;
  if (exp == 0) {
    if (man == 0) bits = sign;
    else {
      exp = 127 - 15 + 1;
      while (!(man & 0x400)) { man <<= 1; exp--; }
      man &= 0x3FF;
      bits = sign | (exp << 23) | (man << 13);
    }
  } else if (exp == 31) {
    bits = sign | 0x7F800000u | (man << 13);
  } else {
    bits = sign | ((exp - 15 + 127) << 23) | (man << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

uint16_t float_to_half_host(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t ax = x & 0x7FFFFFFFu;
  if (ax >= 0x7F800000u) return (uint16_t)(sign | 0x7C00u | (ax > 0x7F800000u ? 0x200u : 0u));  // inf / nan
  if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);                                    // rounds to inf
  if (ax < 0x38800000u) {  // subnormal half (or zero): value = m * 2^-24
    if (ax < 0x33000000u) return (uint16_t)sign;                 // < 2^-25: rounds to 0
    const uint32_t e = ax >> 23, m = (ax & 0x7FFFFFu) | 0x800000u;
    const int shift = 126 - (int)e;                              // 14 .. 24
    uint32_t h = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((ax >> 13) - (112u << 10));  // rebias exponent 127 -> 15
  const uint32_t rem = ax & 0x1FFFu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
  return (uint16_t)(sign | h);
}

namespace {
struct Cursor {
  const uint8_t* p;
  const uint8_t* end;
  template <class T>
  T get() {
    if (p + sizeof(T) > end) throw std::runtime_error("truncated");
    T v;
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    uint64_t n = get<uint64_t>();
    if (p + n > end) throw std::runtime_error("truncated string");
    std::string s((const char*)p, n);
    p += n;
    return s;
  }
};

void read_scalar(Cursor& c, uint32_t t, GGUFValue& v) {
  switch (t) {
    case 0: v.i = c.get<uint8_t>(); break;
    case 1: v.i = c.get<int8_t>(); break;
    case 2: v.i = c.get<uint16_t>(); break;
    case 3: v.i = c.get<int16_t>(); break;
    case 4: v.i = c.get<uint32_t>(); break;
    case 5: v.i = c.get<int32_t>(); break;
    case 6: v.f = c.get<float>(); break;
    case 7: v.i = c.get<uint8_t>(); break;
    case 8: v.s = c.str(); break;
    case 10: v.i = (int64_t)c.get<uint64_t>(); break;
    case 11: v.i = c.get<int64_t>(); break;
    case 12: v.f = c.get<double>(); break;
    default: throw std::runtime_error("bad kv type");
  }
}
}  // namespace

GGUFFile::~GGUFFile() {
  if (map) munmap((void*)map, map_size);
}

bool GGUFFile::open(const std::string& path) {
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) {
    g_gguf_err = "open failed: " + path;
    return false;
  }
  struct stat st;
  fstat(fd, &st);
  map_size = (size_t)st.st_size;
  void* m = mmap(nullptr, map_size, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) {
    g_gguf_err = "mmap failed";
    map = nullptr;
    return false;
  }
  map = (const uint8_t*)m;
  try {
    Cursor c{map, map + map_size};
    if (c.get<uint32_t>() != 0x46554747u) throw std::runtime_error("bad magic");  // "GGUF"
    version = c.get<uint32_t>();
    if (version < 2) throw std::runtime_error("unsupported GGUF version");
    const uint64_t n_tensors = c.get<uint64_t>(), n_kv = c.get<uint64_t>();
    for (uint64_t i = 0; i < n_kv; ++i) {
      std::string key = c.str();
      GGUFValue v;
      v.type = c.get<uint32_t>();
      if (v.type == 9) {
        uint32_t at = c.get<uint32_t>();
        uint64_t n = c.get<uint64_t>();
        for (uint64_t j = 0; j < n; ++j) {
          GGUFValue e;
          read_scalar(c, at, e);
          if (at == 8) v.arr_s.push_back(std::move(e.s));
          else if (at == 6 || at == 12) v.arr_f.push_back(e.f);
          else v.arr_i.push_back(e.i);
        }
      } else {
        read_scalar(c, v.type, v);
      }
      if (key == "general.alignment") alignment = (uint64_t)v.i;
      kv[key] = std::move(v);
    }
    for (uint64_t i = 0; i < n_tensors; ++i) {
      GGUFTensor t;
      t.name = c.str();
      uint32_t nd = c.get<uint32_t>();
      t.n_elements = 1;
      for (uint32_t j = 0; j < nd; ++j) {
        t.dims.push_back((int64_t)c.get<uint64_t>());
        t.n_elements *= t.dims.back();
      }
      t.type = c.get<uint32_t>();
      t.offset = c.get<uint64_t>();
      if (t.type == GGML_F32) t.n_bytes = t.n_elements * 4;
      else if (t.type == GGML_F16) t.n_bytes = t.n_elements * 2;
      else if (t.type == GGML_Q8_0) t.n_bytes = t.n_elements / 32 * 34;
      else t.n_bytes = -1;
      tensors.push_back(std::move(t));
    }
    const uint64_t pos = (uint64_t)(c.p - map);
    data_offset = (pos + alignment - 1) / alignment * alignment;
    for (const auto& t : tensors)
      if (t.n_bytes > 0 && data_offset + t.offset + (uint64_t)t.n_bytes > map_size)
        throw std::runtime_error("tensor data out of file: " + t.name);
  } catch (std::exception& e) {
    g_gguf_err = e.what();
    return false;
  }
  return true;
}

}  // namespace fa
