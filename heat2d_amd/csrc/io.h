// heat2d_amd — output formats.
//
//   * raw binary: native-endian fp32, C-order NX×NY, no header (initial_binary.dat /
//     final_binary.dat, grad1612_mpi_heat.c:177-190,282-285).  Every rank writes its own tile
//     rows with pwrite at ((gx0+i)*NY + gy0)*4 — the correct global file the reference's
//     MPI-IO intended (its final write lacks File_set_view, B-3) — and the file is truncated
//     first (B-9).
//   * "grad" text: NX lines of NY "%6.1f " values (trailing space), row-major
//     (grad1612_mpi_heat.c:191-203,286-298).
//   * "heat2dn" text: transposed, for iy = NY-1..0 a line of NX "%6.1f" values separated by
//     single spaces (mpi_heat2Dn.c:253-268).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace h2d {

enum TextStyle : int { kTextGrad = 0, kTextHeat2dn = 1 };

void binary_create(const std::string& path, int64_t NX, int64_t NY);
void binary_write_tile(const std::string& path, int64_t NX, int64_t NY, int64_t gx0, int64_t gy0, int64_t xcell,
                       int64_t ycell, const float* data);
std::vector<float> binary_read(const std::string& path, int64_t NX, int64_t NY);
void binary_to_text(const std::string& bin, const std::string& txt, int64_t NX, int64_t NY, int style);
std::string format_text(const float* grid, int64_t NX, int64_t NY, int style);

}  // namespace h2d
