// Halo plan of the S-deep exchanges between LDS multi-step passes on a 3-D block decomposition.
//
// A pass of s steps on rank r reads u^{n+S} (out2 of the previous pass) s nodes and u^{n+S−1} (out1) s−1 nodes beyond
// r's box on every side that has a neighbour, corners included (the (y,z) tiles and the x march both reach diagonally).
// MI355X nodes are fully connected (every peer one xGMI hop away), so the corner and edge regions go straight to their
// diagonal neighbours in the same round as the faces: one ncclGroup of at most 26 peers per exchange instead of three
// serialised axis-by-axis rounds (the usual trick on a torus/mesh, where diagonals cost extra hops). Each peer gets ONE
// message: its u^{n+S} region followed by its u^{n+S−1} region, packed contiguously (kernels_halo.hip k_box_copy).
//
// Reference: the block decomposition with face exchange of report.pdf p.4 §1 / SURVEY.md §2.3 C10-C11 (one ghost
// layer per step there); here one exchange every S steps of S-deep ghosts.
#pragma once

#include <array>
#include <vector>

#include "wave3d/cpu.hpp"
#include "wave3d/decomp.hpp"

namespace wave3d {

struct DeepPart {
  int field = 0;  // 0: u^{n+S} (s deep), 1: u^{n+S−1} (s−1 deep)
  LBox send;      // owned nodes next to the face/edge/corner (local indices)
  LBox recv;      // the ghost nodes beyond it (local indices)
  i64 off = 0;    // offset (doubles) of this part inside the peer message
};

struct DeepPeer {
  int peer = -1;
  std::array<int, 3> dir{};  // direction from this rank to the peer, each in {-1, 0, 1}
  i64 count = 0;             // doubles in the message (both directions have the same size)
  i64 buf_off = 0;           // offset of the message in the send / receive staging buffers
  std::vector<DeepPart> parts;
};

struct DeepPlan {
  int s = 0;
  std::vector<DeepPeer> peers;
  i64 total = 0;  // doubles per staging buffer
};

// Plan of the exchange that precedes a pass of `s` steps (2 ≤ s ≤ ghost depth of every split axis). Peers in the order
// of their direction index (dx, dy, dz lexicographic): both ends of a pair see the same single message.
inline DeepPlan make_deep_plan(const Layout& l, const Dims& d, int rank, int s) {
  DeepPlan pl;
  pl.s = s;
  const auto c = rank_coords(d, rank);
  const int lim[3] = {d.px, d.py, d.pz};
  const i64 n[3] = {l.nx, l.ny, l.nz};
  for (int dx = -1; dx <= 1; ++dx)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dz = -1; dz <= 1; ++dz) {
        if (dx == 0 && dy == 0 && dz == 0) continue;
        const int dd[3] = {dx, dy, dz};
        int q[3];
        bool ok = true;
        for (int a = 0; a < 3; ++a) {
          q[a] = c[a] + dd[a];
          ok = ok && q[a] >= 0 && q[a] < lim[a];
        }
        if (!ok) continue;
        DeepPeer p;
        p.peer = coords_rank(d, q[0], q[1], q[2]);
        p.dir = {dx, dy, dz};
        for (int f = 0; f < 2; ++f) {
          const i64 w = f == 0 ? s : s - 1;
          if (w <= 0) continue;
          i64 sb[3][2], rb[3][2];
          for (int a = 0; a < 3; ++a) {
            if (dd[a] < 0) {
              sb[a][0] = 0, sb[a][1] = w, rb[a][0] = -w, rb[a][1] = 0;
            } else if (dd[a] > 0) {
              sb[a][0] = n[a] - w, sb[a][1] = n[a], rb[a][0] = n[a], rb[a][1] = n[a] + w;
            } else {
              sb[a][0] = 0, sb[a][1] = n[a], rb[a][0] = 0, rb[a][1] = n[a];
            }
          }
          DeepPart part;
          part.field = f;
          part.send = LBox{sb[0][0], sb[0][1], sb[1][0], sb[1][1], sb[2][0], sb[2][1]};
          part.recv = LBox{rb[0][0], rb[0][1], rb[1][0], rb[1][1], rb[2][0], rb[2][1]};
          part.off = p.count;
          p.count += part.send.count();
          p.parts.push_back(part);
        }
        p.buf_off = pl.total;
        pl.total += round_up(p.count, 32);  // 256-B aligned messages
        pl.peers.push_back(p);
      }
  return pl;
}

}  // namespace wave3d
