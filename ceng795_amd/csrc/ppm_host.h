// Host side of the photon-mapping path: the PPM scene dialect's loader and the flattened,
// reference-identical acceleration structures (untimed, like PPM's Scene constructor).
#ifndef CENG795_PPM_HOST_H_
#define CENG795_PPM_HOST_H_

#include <string>
#include <vector>

#include "ppm_internal.h"

namespace ppm {

struct HostCamera {
  PCamera cam;
  std::string image_name;
  bool photographic_tmo = false;
  float tmo_key = 0.18f, tmo_saturation_percentage = 1.0f, tmo_saturation = 1.0f;
};

struct HostPPM {
  float eps = 0.001f;
  int per_iteration = 8000, iterations = 1000, max_depth = 20;
  std::vector<HostCamera> cameras;
  std::vector<PMaterial> materials;
  std::vector<float> vpos, vnormal;  // 3 per vertex
  std::vector<float> lights;         // 6 per PointLight: position, intensity
  std::vector<PNode> top_nodes, mesh_nodes;
  std::vector<PObject> objects;
  std::vector<PTriangle> triangles;
  std::vector<PMesh> meshes;
  int top_root = 0;
  int top_depth = 0, mesh_depth = 0;  // node levels (stack sizing)
};

// PPM/src/Scene.cpp:373-505 and the loaders it calls; throws std::runtime_error /
// std::ios_base::failure / std::domain_error (features the reference itself leaves empty:
// binary or PLY vertex / face files).
void load_ppm_xml(const std::string& path, HostPPM& out);

}  // namespace ppm

#endif
