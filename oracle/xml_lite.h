// ORACLE TEST INFRASTRUCTURE — a small DOM reader shared by the CPU restatements
// (cpu_ref.cpp for HW2, ppm_ref.cpp for PPM).  tinyxml2 semantics the loaders rely on:
// GetText() is the element's first child when that child is text; Attribute() is NULL when
// the attribute is absent.
#ifndef CENG795_ORACLE_XML_LITE_H_
#define CENG795_ORACLE_XML_LITE_H_
#include <cctype>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace oracle_xml {

struct Elem {
  std::string name;
  std::string text;
  bool has_text = false;
  std::vector<std::pair<std::string, std::string>> attrs;
  const char* attr(const char* n) const {  // tinyxml2 Attribute(): NULL when absent
    for (auto& a : attrs)
      if (a.first == n) return a.second.c_str();
    return nullptr;
  }
  std::vector<std::unique_ptr<Elem>> kids;
  const Elem* child(const char* n) const {
    for (auto& k : kids)
      if (k->name == n) return k.get();
    return nullptr;
  }
  std::vector<const Elem*> all(const char* n) const {
    std::vector<const Elem*> v;
    for (auto& k : kids)
      if (k->name == n) v.push_back(k.get());
    return v;
  }
};

struct XmlParser {
  const std::string& s;
  size_t p = 0;
  explicit XmlParser(const std::string& str) : s(str) {}
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("xml: ") + m); }
  void skip_misc() {
    for (;;) {
      while (p < s.size() && isspace((unsigned char)s[p])) p++;
      if (s.compare(p, 4, "<!--") == 0) {
        size_t e = s.find("-->", p + 4);
        if (e == std::string::npos) fail("unterminated comment");
        p = e + 3;
      } else if (s.compare(p, 2, "<?") == 0) {
        size_t e = s.find("?>", p + 2);
        if (e == std::string::npos) fail("unterminated declaration");
        p = e + 2;
      } else if (s.compare(p, 2, "<!") == 0) {
        size_t e = s.find('>', p + 2);
        if (e == std::string::npos) fail("unterminated doctype");
        p = e + 1;
      } else {
        return;
      }
    }
  }
  static std::string decode(const std::string& t) {
    std::string o;
    for (size_t i = 0; i < t.size(); i++) {
      if (t[i] != '&') {
        o += t[i];
        continue;
      }
      size_t e = t.find(';', i);
      if (e == std::string::npos) {
        o += t[i];
        continue;
      }
      std::string ent = t.substr(i + 1, e - i - 1);
      if (ent == "lt") o += '<';
      else if (ent == "gt") o += '>';
      else if (ent == "amp") o += '&';
      else if (ent == "quot") o += '"';
      else if (ent == "apos") o += '\'';
      else if (!ent.empty() && ent[0] == '#') o += (char)std::strtol(ent.c_str() + 1 + (ent[1] == 'x'), nullptr, ent[1] == 'x' ? 16 : 10);
      else o += "&" + ent + ";";
      i = e;
    }
    return o;
  }
  std::unique_ptr<Elem> element() {
    if (p >= s.size() || s[p] != '<') fail("expected element");
    p++;
    size_t b = p;
    while (p < s.size() && !isspace((unsigned char)s[p]) && s[p] != '>' && s[p] != '/') p++;
    auto e = std::make_unique<Elem>();
    e->name = s.substr(b, p - b);
    // attributes (the HW2 loader ignores them; PPM reads a few)
    while (p < s.size() && s[p] != '>' && !(s[p] == '/' && p + 1 < s.size() && s[p + 1] == '>')) {
      if (isspace((unsigned char)s[p])) {
        p++;
        continue;
      }
      size_t nb = p;
      while (p < s.size() && s[p] != '=' && !isspace((unsigned char)s[p]) && s[p] != '>' &&
             s[p] != '/')
        p++;
      std::string an = s.substr(nb, p - nb);
      while (p < s.size() && isspace((unsigned char)s[p])) p++;
      if (p < s.size() && s[p] == '=') {
        p++;
        while (p < s.size() && isspace((unsigned char)s[p])) p++;
        if (p < s.size() && (s[p] == '"' || s[p] == '\'')) {
          char q = s[p++];
          size_t vb = p;
          while (p < s.size() && s[p] != q) p++;
          e->attrs.emplace_back(an, decode(s.substr(vb, p - vb)));
          p++;
          continue;
        }
      }
      if (an.empty()) p++;
    }
    if (p >= s.size()) fail("unterminated tag");
    if (s[p] == '/') {
      p += 2;
      return e;
    }
    p++;
    bool first = true;
    for (;;) {
      if (p >= s.size()) fail("unterminated element");
      if (s.compare(p, 2, "</") == 0) {
        size_t c = s.find('>', p);
        if (c == std::string::npos) fail("bad close tag");
        p = c + 1;
        return e;
      }
      if (s.compare(p, 4, "<!--") == 0) {
        size_t c = s.find("-->", p);
        if (c == std::string::npos) fail("unterminated comment");
        p = c + 3;
        first = false;
        continue;
      }
      if (s.compare(p, 9, "<![CDATA[") == 0) {
        size_t c = s.find("]]>", p);
        if (c == std::string::npos) fail("unterminated CDATA");
        if (first) {
          e->text = s.substr(p + 9, c - p - 9);
          e->has_text = true;
        }
        first = false;
        p = c + 3;
        continue;
      }
      if (s[p] == '<') {
        e->kids.push_back(element());
        first = false;
        continue;
      }
      size_t c = s.find('<', p);
      if (c == std::string::npos) fail("unterminated text");
      if (first) {
        e->text = decode(s.substr(p, c - p));
        e->has_text = true;
      }
      first = false;
      p = c;
    }
  }
};

}  // namespace oracle_xml
#endif
