/* meshio.h -- OBJ / PLY triangle meshes for the host scene loader (see meshio.cpp). */
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "transform.h"

namespace mi {

/* world-space mesh attributes exactly as Mesh stores them after its constructor */
struct MeshData {
    std::vector<float> pos, nrm, uv;   /* nrm / uv empty when absent */
    std::vector<uint32_t> faces;
};

MeshData load_obj(const std::string &path, const Transform4f &to_world, bool face_normals, bool flip_tex_coords);
MeshData load_ply(const std::string &path, const Transform4f &to_world, bool face_normals, bool flip_tex_coords);
void recompute_vertex_normals(MeshData &m);

} // namespace mi
