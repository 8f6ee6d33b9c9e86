// tiktoken-compatible byte-pair merge core (Llama-3 tokenizer), pybind11 module `_bpe`.
//
// Replaces tiktoken's Rust core used by the reference (jax_llama/llama3_tokenizer.py:58,78-83).
// For each pre-tokenised piece: whole-piece rank lookup, else start from single bytes and
// repeatedly merge the adjacent pair with the lowest rank (ties: leftmost) until no adjacent
// pair is mergeable. O(n^2) per piece like tiktoken's small-piece path; pieces are short
// (regex pre-tokeniser), and a linked "min-rank cache" keeps it to one rank lookup per
// boundary per merge.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

struct SVHash {
  size_t operator()(std::string_view s) const noexcept {
    // FNV-1a 64
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) { h ^= c; h *= 1099511628211ull; }
    return static_cast<size_t>(h);
  }
};

class BPE {
 public:
  void load(const std::vector<py::bytes>& toks, const std::vector<int>& ranks) {
    if (toks.size() != ranks.size()) throw std::runtime_error("tokens/ranks size mismatch");
    storage_.clear();
    storage_.reserve(toks.size());
    for (const auto& t : toks) storage_.emplace_back(std::string(t));
    map_.clear();
    map_.reserve(storage_.size() * 2);
    for (size_t i = 0; i < storage_.size(); ++i) map_.emplace(std::string_view(storage_[i]), ranks[i]);
  }

  size_t size() const { return map_.size(); }

  int rank_of(std::string_view s) const {
    auto it = map_.find(s);
    return it == map_.end() ? INT_MAX : it->second;
  }

  void encode_piece(std::string_view piece, std::vector<int>& out) const {
    const int whole = rank_of(piece);
    if (whole != INT_MAX) { out.push_back(whole); return; }
    const size_t n = piece.size();
    if (n == 0) return;
    // parts[i] = start offset of part i; ranks_[i] = rank of merging part i with part i+1
    std::vector<size_t> start(n + 1);
    for (size_t i = 0; i <= n; ++i) start[i] = i;
    std::vector<int> pr(n + 1, INT_MAX);
    auto pair_rank = [&](size_t i) -> int {  // rank of parts i..i+1 merged
      if (i + 2 >= start.size()) return INT_MAX;
      return rank_of(piece.substr(start[i], start[i + 2] - start[i]));
    };
    for (size_t i = 0; i + 2 < start.size(); ++i) pr[i] = pair_rank(i);
    while (start.size() > 2) {
      int best = INT_MAX;
      size_t bi = 0;
      for (size_t i = 0; i + 2 < start.size(); ++i) {
        if (pr[i] < best) { best = pr[i]; bi = i; }
      }
      if (best == INT_MAX) break;
      start.erase(start.begin() + bi + 1);
      pr.erase(pr.begin() + bi + 1);
      pr[bi] = pair_rank(bi);
      if (bi > 0) pr[bi - 1] = pair_rank(bi - 1);
    }
    for (size_t i = 0; i + 1 < start.size(); ++i) {
      const int r = rank_of(piece.substr(start[i], start[i + 1] - start[i]));
      if (r == INT_MAX) throw std::runtime_error("byte not in rank table");
      out.push_back(r);
    }
  }

  std::vector<int> encode_pieces(const std::vector<py::bytes>& pieces) const {
    std::vector<int> out;
    out.reserve(pieces.size() * 2);
    for (const auto& p : pieces) {
      std::string_view sv = static_cast<std::string_view>(p);
      encode_piece(sv, out);
    }
    return out;
  }

 private:
  std::vector<std::string> storage_;
  std::unordered_map<std::string_view, int, SVHash> map_;
};

// Python str.isspace() for one code point (Unicode White_Space as CPython classifies it).
bool is_space(char32_t c) {
  if (c == 0x20 || (c >= 0x09 && c <= 0x0d) || (c >= 0x1c && c <= 0x1f)) return true;
  if (c < 0x85) return false;
  return c == 0x85 || c == 0xa0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200a) || c == 0x2028 || c == 0x2029 ||
         c == 0x202f || c == 0x205f || c == 0x3000;
}

// Boundaries (code-point offsets, ascending, including 0 and len) that cut `text` into windows of at most
// `window` code points, and cut every maximal run of same-class characters (whitespace / non-whitespace)
// inside a window at offsets run_start + k * max_run (k >= 1). This is the Llama-3 tokenizer's guard
// against pathological inputs (reference llama3_tokenizer.py:131-146,178-202: 400k-char windows,
// 25k-char same-class runs); the pieces between boundaries are encoded independently.
std::vector<size_t> chunk_bounds(const std::u32string& text, size_t window, size_t max_run) {
  std::vector<size_t> cuts{0};
  const size_t n = text.size();
  for (size_t w0 = 0; w0 < n; w0 += window) {
    const size_t w1 = std::min(n, w0 + window);
    if (w0 > 0) cuts.push_back(w0);
    size_t a = w0;  // start of the current same-class run
    while (a < w1) {
      const bool sp = is_space(text[a]);
      size_t b = a + 1;
      while (b < w1 && is_space(text[b]) == sp) ++b;
      for (size_t c = a + max_run; c < b; c += max_run) cuts.push_back(c);
      a = b;
    }
  }
  if (n > 0) cuts.push_back(n);
  return cuts;
}

}  // namespace

PYBIND11_MODULE(_bpe, m) {
  m.def("chunk_bounds", &chunk_bounds, py::arg("text"), py::arg("window"), py::arg("max_run"));
  m.def("is_space", [](const std::u32string& c) { return c.size() == 1 && is_space(c[0]); });
  m.doc() = "jax_llama_amd tiktoken-compatible BPE merge core";
  py::class_<BPE>(m, "BPE")
      .def(py::init<>())
      .def("load", &BPE::load)
      .def("size", &BPE::size)
      .def("encode_pieces", &BPE::encode_pieces)
      .def("encode_piece", [](const BPE& b, const py::bytes& p) {
        std::vector<int> out;
        b.encode_piece(static_cast<std::string_view>(p), out);
        return out;
      });
}
