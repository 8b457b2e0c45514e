// Host runtime pieces that the reference delegated to Rust/C++ libraries:
//   SafeTensors : mmap'd safetensors reader with zero-copy tensor views and TP row/col slicing (D6)
//   faiss I/O   : IndexFlatL2 "IxF2" reader/writer with atomic replace (D4 file format)
//   BlockManager: paged KV-cache block allocator (64-token blocks, block 0 = graph scratch)
#include "runtime.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace ragk_rt {

// ---------------------------------------------------------------------------- SafeTensors
SafeTensors::SafeTensors(const std::string& path) : path_(path) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) throw std::runtime_error("cannot open " + path);
  struct stat st;
  if (fstat(fd_, &st) != 0) throw std::runtime_error("fstat failed: " + path);
  size_ = (size_t)st.st_size;
  if (size_ < 8) throw std::runtime_error("file too small: " + path);
  base_ = (const char*)mmap(nullptr, size_, PROT_READ, MAP_SHARED, fd_, 0);
  if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed: " + path);
  madvise((void*)base_, size_, MADV_SEQUENTIAL);
  uint64_t hlen;
  std::memcpy(&hlen, base_, 8);
  if (8 + hlen > size_) throw std::runtime_error("corrupt safetensors header: " + path);
  const Json h = JsonParser(base_ + 8, (size_t)hlen).parse();
  data_ = base_ + 8 + hlen;
  for (auto& kv : h.obj) {
    if (kv.first == "__metadata__") {
      for (auto& m : kv.second.obj) metadata_[m.first] = m.second.str;
      continue;
    }
    TensorInfo t;
    t.name = kv.first;
    t.dtype = kv.second.at("dtype").str;
    for (auto& d : kv.second.at("shape").arr) t.shape.push_back(d.as_int());
    const Json& off = kv.second.at("data_offsets");
    t.begin = (size_t)off.arr.at(0).as_int();
    t.end = (size_t)off.arr.at(1).as_int();
    if (data_ + t.end > base_ + size_) throw std::runtime_error("tensor out of file bounds: " + t.name);
    order_.push_back(t.name);
    tensors_[t.name] = t;
  }
}

SafeTensors::~SafeTensors() {
  if (base_ && base_ != MAP_FAILED) munmap((void*)base_, size_);
  if (fd_ >= 0) ::close(fd_);
}

size_t dtype_size(const std::string& dt) {
  if (dt == "F64" || dt == "I64" || dt == "U64") return 8;
  if (dt == "F32" || dt == "I32" || dt == "U32") return 4;
  if (dt == "BF16" || dt == "F16" || dt == "I16" || dt == "U16") return 2;
  return 1;
}

const TensorInfo& SafeTensors::info(const std::string& name) const {
  auto it = tensors_.find(name);
  if (it == tensors_.end()) throw std::out_of_range("no tensor " + name);
  return it->second;
}

// copy rows [r0,r1) x cols [c0,c1) of a 2-D tensor (or rows of any-rank tensor when c0<0)
void SafeTensors::copy_slice(const std::string& name, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                             char* dst) const {
  const TensorInfo& t = info(name);
  const size_t es = dtype_size(t.dtype);
  const char* src = data_ + t.begin;
  int64_t row_elems = 1;
  for (size_t i = 1; i < t.shape.size(); ++i) row_elems *= t.shape[i];
  if (t.shape.empty()) {
    std::memcpy(dst, src, es);
    return;
  }
  if (r0 < 0) { r0 = 0; r1 = t.shape[0]; }
  if (c0 < 0) {
    std::memcpy(dst, src + (size_t)r0 * row_elems * es, (size_t)(r1 - r0) * row_elems * es);
    return;
  }
  if (t.shape.size() != 2) throw std::runtime_error("column slicing needs a 2-D tensor: " + name);
  const size_t w = (size_t)(c1 - c0) * es;
  for (int64_t r = r0; r < r1; ++r) std::memcpy(dst + (size_t)(r - r0) * w, src + ((size_t)r * row_elems + c0) * es, w);
}

// ---------------------------------------------------------------------------- faiss IndexFlatL2
FlatIndexData read_flat_index(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  FlatIndexData r;
  char fourcc[4];
  auto rd = [&](void* p, size_t n) {
    if (fread(p, 1, n, f) != n) {
      fclose(f);
      throw std::runtime_error("truncated faiss index file " + path);
    }
  };
  rd(fourcc, 4);
  if (std::memcmp(fourcc, "IxF2", 4) && std::memcmp(fourcc, "IxFI", 4) && std::memcmp(fourcc, "IxFl", 4)) {
    fclose(f);
    throw std::runtime_error("not an IndexFlat file: " + path);
  }
  int32_t d;
  int64_t ntotal, dummy;
  uint8_t trained;
  int32_t metric;
  rd(&d, 4); rd(&ntotal, 8); rd(&dummy, 8); rd(&dummy, 8); rd(&trained, 1); rd(&metric, 4);
  if (metric > 1) { float arg; rd(&arg, 4); }
  uint64_t nf;
  rd(&nf, 8);
  if (nf != (uint64_t)ntotal * (uint64_t)d) {
    fclose(f);
    throw std::runtime_error("corrupt IndexFlat payload size");
  }
  r.d = d;
  r.ntotal = ntotal;
  r.metric = metric;
  r.xb.resize(nf);
  if (nf) rd(r.xb.data(), nf * 4);
  fclose(f);
  return r;
}

void write_flat_index(const std::string& path, const float* xb, int64_t n, int32_t d) {
  const std::string tmp = path + ".tmp." + std::to_string(getpid());
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write " + tmp);
  const int64_t dummy = 1 << 20;
  const uint8_t trained = 1;
  const int32_t metric = 1;
  const uint64_t nf = (uint64_t)n * (uint64_t)d;
  bool ok = fwrite("IxF2", 1, 4, f) == 4 && fwrite(&d, 4, 1, f) == 1 && fwrite(&n, 8, 1, f) == 1 &&
            fwrite(&dummy, 8, 1, f) == 1 && fwrite(&dummy, 8, 1, f) == 1 && fwrite(&trained, 1, 1, f) == 1 &&
            fwrite(&metric, 4, 1, f) == 1 && fwrite(&nf, 8, 1, f) == 1;
  if (ok && nf) ok = fwrite(xb, 4, nf, f) == nf;
  ok = ok && fflush(f) == 0 && fsync(fileno(f)) == 0;
  fclose(f);
  if (!ok || rename(tmp.c_str(), path.c_str()) != 0) {
    unlink(tmp.c_str());
    throw std::runtime_error("failed writing " + path);
  }
}

// ---------------------------------------------------------------------------- BlockManager
BlockManager::BlockManager(int num_blocks, bool reserve_scratch) : num_blocks_(num_blocks) {
  if (num_blocks < 2) throw std::invalid_argument("need at least 2 KV blocks");
  const int first = reserve_scratch ? 1 : 0;
  free_.reserve(num_blocks);
  for (int b = num_blocks - 1; b >= first; --b) free_.push_back(b);
}

int BlockManager::blocks_needed(int64_t seq, int64_t n_tokens) const {
  auto it = tables_.find(seq);
  const int have = it == tables_.end() ? 0 : (int)it->second.size();
  const int need = (int)((n_tokens + kBlock - 1) / kBlock);
  return need > have ? need - have : 0;
}

const std::vector<int>& BlockManager::ensure(int64_t seq, int64_t n_tokens) {
  std::vector<int>& t = tables_[seq];
  const size_t need = (size_t)((n_tokens + kBlock - 1) / kBlock);
  if (need > t.size() && need - t.size() > free_.size()) throw std::runtime_error("KV cache exhausted");
  while (t.size() < need) {
    t.push_back(free_.back());
    free_.pop_back();
  }
  return t;
}

const std::vector<int>& BlockManager::table(int64_t seq) const {
  static const std::vector<int> empty;
  auto it = tables_.find(seq);
  return it == tables_.end() ? empty : it->second;
}

void BlockManager::free(int64_t seq) {
  auto it = tables_.find(seq);
  if (it == tables_.end()) return;
  for (auto b = it->second.rbegin(); b != it->second.rend(); ++b) free_.push_back(*b);
  tables_.erase(it);
}

}  // namespace ragk_rt
