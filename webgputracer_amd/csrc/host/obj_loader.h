// obj_loader.h — Wavefront OBJ reader replacing tinyobjloader (an empty, unpinned
// submodule in the reference, .gitmodules:4-5) for Scene::LoadVertices
// (scene.cpp:70-131): one Vertex per face corner, normal defaulting to (0,0,1) and
// uv to (0,0) (scene.cpp:101-105), faces with n > 3 corners fan-triangulated
// (v0, vi, vi+1) the way tinyobjloader's default triangulation emits them.
#pragma once

#include <string>
#include <vector>

#include "../../../include/wgt/objects.h"

namespace wgt {
namespace obj {
bool LoadTriangulated(const char* path, std::vector<Vertex>& vertices, std::string& err,
                      std::string& warn);
bool ParseTriangulated(const std::string& text, std::vector<Vertex>& vertices, std::string& err,
                       std::string& warn);
}  // namespace obj
}  // namespace wgt
