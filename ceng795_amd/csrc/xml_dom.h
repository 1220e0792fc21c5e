// Small XML DOM reader for the scene loaders (HW2 dialect: scene_xml.cpp; PPM dialect:
// ppm_scene.cpp).  Covers what the scene files use: elements, attributes, text, CDATA,
// comments, processing instructions, the five predefined entities and numeric character
// references.  tinyxml2 semantics the loaders rely on: GetText() is the element's first child
// when that child is text; Attribute() is NULL when absent; the document's FIRST node is the
// scene root, so a leading <?xml?> declaration or comment makes the file unloadable, as in the
// reference — here an error instead of the reference's crash.
#ifndef CENG795_XML_DOM_H_
#define CENG795_XML_DOM_H_

#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace rt {

struct Node {
  std::string tag;
  std::string text;
  bool has_text = false;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<std::unique_ptr<Node>> children;
  const Node* first(const char* name) const {
    for (const auto& c : children)
      if (c->tag == name) return c.get();
    return nullptr;
  }
  std::vector<const Node*> each(const char* name) const {
    std::vector<const Node*> r;
    for (const auto& c : children)
      if (c->tag == name) r.push_back(c.get());
    return r;
  }
  const char* attr(const char* name) const {
    for (const auto& a : attrs)
      if (a.first == name) return a.second.c_str();
    return nullptr;
  }
  int int_attr(const char* name, int fallback) const;    // tinyxml2 IntAttribute
  bool bool_attr(const char* name, bool fallback) const; // tinyxml2 BoolAttribute
};

// Parses a whole file; throws std::ios_base::failure (unreadable) / std::runtime_error.
std::unique_ptr<Node> parse_xml_file(const std::string& path);
// Text of an element; throws std::runtime_error naming `what` when missing.
const char* node_text(const Node* n, const char* what);

}  // namespace rt

#endif
