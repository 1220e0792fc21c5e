// XML DOM reader (see xml_dom.h).
#include "xml_dom.h"

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <ios>
#include <iterator>
#include <stdexcept>

namespace rt {
namespace {


class Reader {
 public:
  explicit Reader(std::string doc) : s_(std::move(doc)) {}

  std::unique_ptr<Node> document_root() {
    // The reference takes XMLDocument::FirstChild() as the scene root (HW2/Scene.cpp:206,
    // PPM/src/Scene.cpp:381): a declaration, comment or DOCTYPE in front of the root element
    // becomes the "root", and the loader then dereferences its missing <Cameras> child.  That
    // file does not load there, so it does not load here either (an error, not a crash).
    while (i_ < s_.size() && std::isspace((unsigned char)s_[i_])) ++i_;
    if (at("<?") || at("<!"))
      error("the first node is not the scene element (a declaration, comment or DOCTYPE; the "
            "reference takes FirstChild() as the root and cannot load this file)");
    if (i_ >= s_.size() || s_[i_] != '<') error("no root element");
    return parse_element();
  }

 private:
  std::string s_;
  size_t i_ = 0;

  [[noreturn]] void error(const std::string& what) const {
    throw std::runtime_error("scene xml: " + what + " at byte " + std::to_string(i_));
  }
  bool at(const char* lit) const { return s_.compare(i_, std::strlen(lit), lit) == 0; }
  void skip_to(const char* end) {
    const size_t k = s_.find(end, i_);
    if (k == std::string::npos) error(std::string("missing ") + end);
    i_ = k + std::strlen(end);
  }
  static std::string unescape(const std::string& raw) {
    std::string out;
    out.reserve(raw.size());
    for (size_t k = 0; k < raw.size(); ++k) {
      if (raw[k] != '&') {
        out.push_back(raw[k]);
        continue;
      }
      const size_t semi = raw.find(';', k);
      if (semi == std::string::npos) {
        out.push_back('&');
        continue;
      }
      const std::string e = raw.substr(k + 1, semi - k - 1);
      if (e == "amp") out.push_back('&');
      else if (e == "lt") out.push_back('<');
      else if (e == "gt") out.push_back('>');
      else if (e == "quot") out.push_back('"');
      else if (e == "apos") out.push_back('\'');
      else if (e.size() > 1 && e[0] == '#') {
        const bool hexa = e[1] == 'x' || e[1] == 'X';
        out.push_back((char)std::strtol(e.c_str() + (hexa ? 2 : 1), nullptr, hexa ? 16 : 10));
      } else {
        out += "&" + e + ";";
      }
      k = semi;
    }
    return out;
  }
  std::unique_ptr<Node> parse_element() {
    ++i_;  // '<'
    const size_t name_begin = i_;
    while (i_ < s_.size() && !std::isspace((unsigned char)s_[i_]) && s_[i_] != '>' &&
           s_[i_] != '/')
      ++i_;
    auto node = std::make_unique<Node>();
    node->tag = s_.substr(name_begin, i_ - name_begin);
    if (node->tag.empty()) error("empty tag name");
    for (;;) {  // attributes: name = "value" | 'value'
      if (i_ >= s_.size()) error("unterminated start tag");
      const char c = s_[i_];
      if (c == '>') {
        ++i_;
        break;
      }
      if (c == '/' && i_ + 1 < s_.size() && s_[i_ + 1] == '>') {
        i_ += 2;
        return node;
      }
      if (std::isspace((unsigned char)c)) {
        ++i_;
        continue;
      }
      const size_t nb = i_;
      while (i_ < s_.size() && s_[i_] != '=' && s_[i_] != '>' && s_[i_] != '/' &&
             !std::isspace((unsigned char)s_[i_]))
        ++i_;
      const std::string name = s_.substr(nb, i_ - nb);
      while (i_ < s_.size() && std::isspace((unsigned char)s_[i_])) ++i_;
      if (name.empty() || i_ >= s_.size() || s_[i_] != '=') {
        if (name.empty()) ++i_;
        continue;
      }
      ++i_;
      while (i_ < s_.size() && std::isspace((unsigned char)s_[i_])) ++i_;
      if (i_ >= s_.size() || (s_[i_] != '"' && s_[i_] != '\'')) error("attribute without quotes");
      const size_t q = s_.find(s_[i_], i_ + 1);
      if (q == std::string::npos) error("unterminated attribute");
      node->attrs.emplace_back(name, unescape(s_.substr(i_ + 1, q - i_ - 1)));
      i_ = q + 1;
    }
    bool first_child = true;
    for (;;) {
      if (i_ >= s_.size()) error("unterminated element <" + node->tag + ">");
      if (at("</")) {
        skip_to(">");
        return node;
      }
      if (at("<!--")) {
        skip_to("-->");
        first_child = false;
        continue;
      }
      if (at("<![CDATA[")) {
        const size_t begin = i_ + 9;
        skip_to("]]>");
        if (first_child) {
          node->text = s_.substr(begin, i_ - 3 - begin);
          node->has_text = true;
        }
        first_child = false;
        continue;
      }
      if (at("<?")) {
        skip_to("?>");
        first_child = false;
        continue;
      }
      if (s_[i_] == '<') {
        node->children.push_back(parse_element());
        first_child = false;
        continue;
      }
      const size_t end = s_.find('<', i_);
      if (end == std::string::npos) error("text runs to end of file");
      if (first_child) {
        node->text = unescape(s_.substr(i_, end - i_));
        node->has_text = true;
      }
      first_child = false;
      i_ = end;
    }
  }
};

}  // namespace

int Node::int_attr(const char* name, int fallback) const {
  const char* a = attr(name);
  if (!a) return fallback;
  int v = fallback;
  return std::sscanf(a, "%d", &v) == 1 ? v : fallback;
}

bool Node::bool_attr(const char* name, bool fallback) const {
  const char* a = attr(name);
  if (!a) return fallback;
  if (!std::strcmp(a, "true") || !std::strcmp(a, "1")) return true;
  if (!std::strcmp(a, "false") || !std::strcmp(a, "0")) return false;
  int v;
  return std::sscanf(a, "%d", &v) == 1 ? v != 0 : fallback;
}

std::unique_ptr<Node> parse_xml_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::ios_base::failure("Error: The xml file cannot be loaded: " + path);
  std::string doc((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  return Reader(std::move(doc)).document_root();
}

const char* node_text(const Node* n, const char* what) {
  if (!n) throw std::runtime_error(std::string("scene xml: missing <") + what + ">");
  if (!n->has_text) throw std::runtime_error(std::string("scene xml: <") + what + "> has no text");
  return n->text.c_str();
}

}  // namespace rt
