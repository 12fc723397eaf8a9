#include "extender_scan.h"

#include <array>
#include <cstring>

namespace kgwe {

namespace {

class Scanner {
 public:
  explicit Scanner(std::string_view t) : t_(t) {}

  void ws() {
    while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\n' || t_[p_] == '\r' || t_[p_] == '\t')) ++p_;
  }
  bool eat(char c) {
    ws();
    if (p_ < t_.size() && t_[p_] == c) {
      ++p_;
      return true;
    }
    return false;
  }
  bool peek(char c) {
    ws();
    return p_ < t_.size() && t_[p_] == c;
  }
  // A string token; `plain` is false when it contains escapes (the raw text
  // between the quotes is returned in that case).
  bool string(std::string_view* s, bool* plain = nullptr) {
    ws();
    if (p_ >= t_.size() || t_[p_] != '"') return false;
    const size_t b = ++p_;
    bool esc = false;
    while (p_ < t_.size()) {
      const char* q = static_cast<const char*>(std::memchr(t_.data() + p_, '"', t_.size() - p_));
      if (!q) return false;
      const size_t at = static_cast<size_t>(q - t_.data());
      // count the backslashes right before the quote
      size_t k = at;
      while (k > b && t_[k - 1] == '\\') --k;
      if (((at - k) & 1) == 0) {
        esc |= std::memchr(t_.data() + b, '\\', at - b) != nullptr;
        *s = t_.substr(b, at - b);
        if (plain) *plain = !esc;
        p_ = at + 1;
        return true;
      }
      p_ = at + 1;
    }
    return false;
  }
  // Skip one JSON value of any type.
  bool skip() {
    ws();
    if (p_ >= t_.size()) return false;
    const char c = t_[p_];
    if (c == '"') {
      std::string_view s;
      return string(&s);
    }
    if (c == '{' || c == '[') {
      // Only quotes and brackets matter inside a container: jump between
      // them with a byte-class table; strings are skipped with memchr.
      static const auto kInteresting = [] {
        std::array<bool, 256> t{};
        for (unsigned char ch : {'"', '{', '}', '[', ']'}) t[ch] = true;
        return t;
      }();
      int depth = 0;
      const char* d = t_.data();
      const size_t n = t_.size();
      size_t i = p_;
      while (i < n) {
        while (i < n && !kInteresting[static_cast<unsigned char>(d[i])]) ++i;
        if (i >= n) break;
        const char ch = d[i];
        if (ch == '"') {
          // end of string: next unescaped quote
          size_t j = i + 1;
          while (true) {
            const char* q = static_cast<const char*>(std::memchr(d + j, '"', n - j));
            if (!q) return false;
            size_t at = static_cast<size_t>(q - d), k = at;
            while (k > i + 1 && d[k - 1] == '\\') --k;
            j = at + 1;
            if (((at - k) & 1) == 0) break;
          }
          i = j;
          continue;
        }
        if (ch == '{' || ch == '[') {
          ++depth;
        } else if (--depth == 0) {
          p_ = i + 1;
          return true;
        }
        ++i;
      }
      return false;
    }
    while (p_ < t_.size() && t_[p_] != ',' && t_[p_] != '}' && t_[p_] != ']' && t_[p_] != ' ' &&
           t_[p_] != '\n' && t_[p_] != '\r' && t_[p_] != '\t')
      ++p_;
    return true;
  }
  size_t pos() const { return p_; }
  void set(size_t p) { p_ = p; }
  std::string_view text() const { return t_; }

 private:
  std::string_view t_;
  size_t p_ = 0;
};

// Inside an object that starts at the scanner position: call f(key) for
// every member with the scanner on the value; f must consume the value.
template <class F>
bool members(Scanner& s, F f) {
  if (!s.eat('{')) return false;
  if (s.eat('}')) return true;
  while (true) {
    std::string_view key;
    if (!s.string(&key) || !s.eat(':')) return false;
    if (!f(key)) return false;
    if (s.eat(',')) continue;
    return s.eat('}');
  }
}

// metadata.name of one Node item (scanner on the item).
bool item_name(Scanner& s, std::string* name) {
  return members(s, [&](std::string_view k) {
    if (k != "metadata") return s.skip();
    return members(s, [&](std::string_view mk) {
      if (mk != "name") return s.skip();
      std::string_view v;
      bool plain = false;
      if (!s.string(&v, &plain) || !plain) return false;
      name->assign(v.data(), v.size());
      return true;
    });
  });
}

bool node_items(Scanner& s, std::vector<NodeSpan>* out) {
  return members(s, [&](std::string_view k) {
    if (k != "items" && k != "Items") return s.skip();
    if (s.eat('[') && !s.eat(']')) {
      while (true) {
        s.ws();
        NodeSpan n;
        n.begin = s.pos();
        if (!item_name(s, &n.name)) return false;
        n.end = s.pos();
        out->push_back(std::move(n));
        if (s.eat(',')) continue;
        return s.eat(']');
      }
    }
    return true;
  });
}

}  // namespace

bool scan_extender_args(std::string_view text, ExtenderArgsScan* out) {
  Scanner s(text);
  return members(s, [&](std::string_view k) {
    if (k == "pod" || k == "Pod") {
      s.ws();
      const size_t b = s.pos();
      if (!s.skip()) return false;
      out->pod = Json::parse(std::string(text.substr(b, s.pos() - b)));
      return true;
    }
    if (k == "nodes" || k == "Nodes") {
      if (s.peek('n')) return s.skip();  // null
      out->have_nodes = true;
      return node_items(s, &out->nodes);
    }
    if (k == "nodenames" || k == "NodeNames") {
      if (s.peek('n')) return s.skip();
      if (!s.eat('[')) return false;
      if (s.eat(']')) return true;
      while (true) {
        std::string_view v;
        bool plain = false;
        if (!s.string(&v, &plain) || !plain) return false;
        out->nodenames.emplace_back(v);
        if (s.eat(',')) continue;
        return s.eat(']');
      }
    }
    return s.skip();
  });
}

bool scan_node_names(std::string_view text, std::vector<std::string>* names) {
  ExtenderArgsScan a;
  try {
    if (!scan_extender_args(text, &a)) return false;
  } catch (...) {
    return false;
  }
  for (auto& n : a.nodes) names->push_back(std::move(n.name));
  for (auto& n : a.nodenames) names->push_back(std::move(n));
  return true;
}

}  // namespace kgwe
