// The product's kernels (timestep.hip) and C-ABI (capi.cpp) compiled for the
// host against the execution-model emulation in hip/hip_runtime.h (test
// infrastructure only): reads a world description and inputs written by
// tests/test_wave_emu.py, runs nimble_forward + nimble_backward through the
// C-ABI exactly as on the GPU, and prints next states, gradients and the
// snapshot headers.  Built with AddressSanitizer: any out-of-bounds access of
// the kernels on these inputs aborts the run with its location.
//
// input (whitespace-separated):
//   nb n ns nmv pen par hasCand   dt g0 g1 g2 clip cfm
//   parent[nb] skeleton[nb] joint_type[nb] dof_offset[nb] mobile[nb]
//   Tp[12nb] Tc[12nb] axis[3nb] mass[nb] com[3nb] moment[6nb] friction[nb] restitution[nb]
//   damping[n] spring[n] rest[n] plo[n] phi[n] vlo[n] vhi[n] flo[n] fhi[n]
//   shape_body[ns] shape_type[ns] shape_size[3ns] shape_T[12ns]
//   mesh_first[ns] mesh_count[ns] mesh_vertices[3nmv] (candidate[nmv] if hasCand)
//   B  state[B 2n]  forces[B n]  grad_next[B 2n]
// environment: NIMBLE_AMD_DEFER_ROWS / NIMBLE_AMD_LDS_ROWS as for the GPU
// output lines: "next" [B 2n], "gs" [B 2n], "gf" [B n], "head" [B 16]
#include <cstdio>
#include <iostream>
#include <string>
#include <vector>

double s[160 * 1024 / 8];  // the workgroup's LDS (dynamic shared memory)

#include "../../../nimblephysics_amd/csrc/timestep.hip"
#include "../../../nimblephysics_amd/csrc/capi.cpp"

template <class T>
static std::vector<T> readArr(size_t n) {
  std::vector<T> v(n);
  for (auto& x : v) {
    std::string t;
    if (!(std::cin >> t)) { std::fprintf(stderr, "short input\n"); std::exit(2); }
    if constexpr (std::is_same<T, double>::value) x = std::strtod(t.c_str(), nullptr);
    else x = (T)std::strtol(t.c_str(), nullptr, 10);
  }
  return v;
}

static void print(const char* key, const std::vector<double>& v) {
  std::printf("%s", key);
  for (double x : v) std::printf(" %.17g", x);
  std::printf("\n");
}

int main() {
  auto hi = readArr<int>(7);
  auto hd = readArr<double>(6);
  const int nb = hi[0], n = hi[1], ns = hi[2], nmv = hi[3];
  auto parent = readArr<int32_t>(nb), skel = readArr<int32_t>(nb), jt = readArr<int32_t>(nb);
  auto dof0 = readArr<int32_t>(nb), mobile = readArr<int32_t>(nb);
  auto Tp = readArr<double>(12 * nb), Tc = readArr<double>(12 * nb), axis = readArr<double>(3 * nb);
  auto mass = readArr<double>(nb), com = readArr<double>(3 * nb), moment = readArr<double>(6 * nb);
  auto fric = readArr<double>(nb), rest = readArr<double>(nb);
  std::vector<std::vector<double>> dofs;
  for (int k = 0; k < 9; k++) dofs.push_back(readArr<double>(n));
  auto sb = readArr<int32_t>(ns), st = readArr<int32_t>(ns);
  auto ssz = readArr<double>(3 * ns), sT = readArr<double>(12 * ns);
  auto mf = readArr<int32_t>(ns), mc = readArr<int32_t>(ns);
  auto mv = readArr<double>(3 * (size_t)nmv);
  std::vector<int32_t> cand;
  if (hi[6]) cand = readArr<int32_t>(nmv);
  nimble_world_desc d{};
  d.num_bodies = nb; d.num_dofs = n; d.num_shapes = ns;
  d.dt = hd[0]; d.gravity[0] = hd[1]; d.gravity[1] = hd[2]; d.gravity[2] = hd[3];
  d.contact_clipping_depth = hd[4]; d.fallback_cfm = hd[5];
  d.penetration_correction = hi[4]; d.parallel_pos_vel = hi[5];
  d.parent = parent.data(); d.skeleton = skel.data(); d.joint_type = jt.data(); d.dof_offset = dof0.data();
  d.skeleton_mobile = mobile.data(); d.T_parent_joint = Tp.data(); d.T_child_joint = Tc.data();
  d.axis = axis.data(); d.mass = mass.data(); d.com = com.data(); d.moment = moment.data();
  d.friction = fric.data(); d.restitution = rest.data();
  d.damping = dofs[0].data(); d.spring = dofs[1].data(); d.rest_position = dofs[2].data();
  d.pos_lower = dofs[3].data(); d.pos_upper = dofs[4].data(); d.vel_lower = dofs[5].data();
  d.vel_upper = dofs[6].data(); d.force_lower = dofs[7].data(); d.force_upper = dofs[8].data();
  d.shape_body = sb.data(); d.shape_type = st.data(); d.shape_size = ssz.data(); d.shape_T = sT.data();
  d.num_mesh_vertices = nmv; d.mesh_vertices = nmv ? mv.data() : nullptr;
  d.shape_mesh_first = mf.data(); d.shape_mesh_count = mc.data();
  d.mesh_vertex_candidate = hi[6] ? cand.data() : nullptr;
  nimble_world_t w = nullptr;
  if (nimble_world_create(&d, &w) != NIMBLE_OK) {
    std::fprintf(stderr, "create: %s\n", nimble_last_error());
    return 3;
  }
  const int B = readArr<int>(1)[0];
  auto state = readArr<double>((size_t)B * 2 * n), forces = readArr<double>((size_t)B * n);
  auto grad = readArr<double>((size_t)B * 2 * n);
  const int64_t sd = nimble_snapshot_doubles(w), cd = nimble_lcp_cache_doubles(w);
  std::vector<double> cache((size_t)B * cd, 0.0), next((size_t)B * 2 * n), snap((size_t)B * sd, 0.0);
  for (int b = 0; b < B; b++) cache[(size_t)b * cd] = -1.0;
  std::vector<double> gs((size_t)B * 2 * n), gf((size_t)B * n);
  if (nimble_forward(w, B, state.data(), forces.data(), cache.data(), next.data(), snap.data(), nullptr) != NIMBLE_OK ||
      nimble_backward(w, B, state.data(), forces.data(), snap.data(), grad.data(), gs.data(), gf.data(), nullptr) !=
          NIMBLE_OK) {
    std::fprintf(stderr, "step: %s\n", nimble_last_error());
    return 4;
  }
  std::vector<double> head;
  for (int b = 0; b < B; b++)
    for (int k = 0; k < 16; k++) head.push_back(snap[(size_t)b * sd + k]);
  print("next", next);
  print("gs", gs);
  print("gf", gf);
  print("head", head);
  nimble_world_destroy(w);
  return 0;
}
