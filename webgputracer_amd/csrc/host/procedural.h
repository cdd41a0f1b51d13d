// procedural.h — deterministic stand-ins for the absent Bunny / Sponza assets
// (*.obj are gitignored by the reference and there is no network).
// Both are placed inside the Cornell box (x, y, z in [0, 555]) so that the
// reference light (scene.cpp:16) illuminates them.
#pragma once

#include <cstdint>
#include <vector>

#include "../../../include/wgt/objects.h"

namespace wgt {
namespace procedural {
// Closed, star-shaped displaced blob with two "ears" (Stanford-bunny-sized:
// ~69k triangles for target 69451), sitting on the floor.
void Bunny(uint32_t target_tris, uint32_t seed, std::vector<Triangle>& out);
// Atrium: tiled floor, two colonnades with arches, gallery slabs and folded
// drapes (Sponza-sized: ~262k triangles for target 262267).
void Sponza(uint32_t target_tris, uint32_t seed, std::vector<Triangle>& out);
}  // namespace procedural
}  // namespace wgt
