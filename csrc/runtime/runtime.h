#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "json.h"

namespace ragk_rt {

struct TensorInfo {
  std::string name, dtype;
  std::vector<int64_t> shape;
  size_t begin = 0, end = 0;
};

size_t dtype_size(const std::string& dt);

class SafeTensors {
 public:
  explicit SafeTensors(const std::string& path);
  ~SafeTensors();
  SafeTensors(const SafeTensors&) = delete;
  SafeTensors& operator=(const SafeTensors&) = delete;
  const std::vector<std::string>& keys() const { return order_; }
  const TensorInfo& info(const std::string& name) const;
  const char* data(const std::string& name) const { return data_ + info(name).begin; }
  void copy_slice(const std::string& name, int64_t r0, int64_t r1, int64_t c0, int64_t c1, char* dst) const;
  const std::map<std::string, std::string>& metadata() const { return metadata_; }

 private:
  std::string path_;
  int fd_ = -1;
  size_t size_ = 0;
  const char* base_ = nullptr;
  const char* data_ = nullptr;
  std::vector<std::string> order_;
  std::unordered_map<std::string, TensorInfo> tensors_;
  std::map<std::string, std::string> metadata_;
};

struct FlatIndexData {
  int32_t d = 0;
  int64_t ntotal = 0;
  int32_t metric = 1;
  std::vector<float> xb;
};
FlatIndexData read_flat_index(const std::string& path);
void write_flat_index(const std::string& path, const float* xb, int64_t n, int32_t d);

class BlockManager {
 public:
  static constexpr int kBlock = 64;
  BlockManager(int num_blocks, bool reserve_scratch);
  int free_blocks() const { return (int)free_.size(); }
  int blocks_needed(int64_t seq, int64_t n_tokens) const;
  bool can_allocate(int64_t seq, int64_t n_tokens) const { return blocks_needed(seq, n_tokens) <= free_blocks(); }
  const std::vector<int>& ensure(int64_t seq, int64_t n_tokens);
  const std::vector<int>& table(int64_t seq) const;
  int64_t slot(int64_t seq, int64_t pos) const { return (int64_t)table(seq).at(pos / kBlock) * kBlock + pos % kBlock; }
  void free(int64_t seq);
  int num_blocks() const { return num_blocks_; }

 private:
  int num_blocks_;
  std::vector<int> free_;
  std::unordered_map<int64_t, std::vector<int>> tables_;
};

}  // namespace ragk_rt
