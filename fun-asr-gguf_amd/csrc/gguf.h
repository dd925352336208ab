// Minimal GGUF v3 reader (mmap): header, metadata KV, tensor infos, aligned data section.
// Format per the vendored gguf-py (gguf/constants.py:10-12 GGUF_MAGIC/VERSION/DEFAULT_ALIGNMENT,
// gguf_reader.py:132-182); replaces llama_model_load_from_file for the decoder weights.
#pragma once
#include <stdint.h>
#include <string>
#include <unordered_map>
#include <vector>

namespace fa {

enum { GGML_F32 = 0, GGML_F16 = 1, GGML_Q8_0 = 8 };

struct GGUFTensor {
  std::string name;
  std::vector<int64_t> dims;
  uint32_t type = 0;
  uint64_t offset = 0;
  int64_t n_elements = 0, n_bytes = 0;
};

struct GGUFValue {
  uint32_t type = 0;
  int64_t i = 0;
  double f = 0;
  std::string s;
  std::vector<std::string> arr_s;
  std::vector<int64_t> arr_i;
  std::vector<double> arr_f;
};

struct GGUFFile {
  std::vector<GGUFTensor> tensors;
  std::unordered_map<std::string, GGUFValue> kv;
  uint32_t version = 0;
  uint64_t alignment = 32, data_offset = 0;
  const uint8_t* map = nullptr;
  size_t map_size = 0;
  bool open(const std::string& path);
  const uint8_t* data(const GGUFTensor& t) const { return map + data_offset + t.offset; }
  ~GGUFFile();
};

const char* gguf_error();
float half_to_float_host(uint16_t h);
uint16_t float_to_half_host(float f);  // IEEE binary16, round to nearest even

}  // namespace fa
