// Field dumps and checkpoints of the native runtime: wave3d-dump-v1 (SURVEY.md §5.9 — the reference writes no field
// at all, report.pdf / readme.md have only stdout). See wave3d/runtime.hpp.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>

#include "wave3d/runtime.hpp"

namespace wave3d {

void write_dump(const std::string& prefix, const Problem& p, const Layout& l, const std::vector<double>& u, int rank,
                int world, const Dims& d, int step) {
  if (step < 0) step = p.K;
  const std::string base = world > 1 ? prefix + ".rank" + std::to_string(rank) : prefix;
  std::ofstream f(base + ".bin", std::ios::binary | std::ios::trunc);
  std::vector<double> row(static_cast<size_t>(l.nz));
  for (i64 ix = 0; ix < l.nx; ++ix)
    for (i64 iy = 0; iy < l.ny; ++iy) {
      const double* src = u.data() + l.off(ix, iy, 0);
      std::memcpy(row.data(), src, row.size() * sizeof(double));
      f.write(reinterpret_cast<const char*>(row.data()), static_cast<std::streamsize>(row.size() * sizeof(double)));
    }
  std::ofstream j(base + ".json", std::ios::trunc);
  j.precision(17);
  j << "{\"format\": \"wave3d-dump-v1\", \"dtype\": \"float64\", \"order\": \"C\", \"N\": " << p.N
    << ", \"L\": " << p.L << ", \"tau\": " << p.tau << ", \"step\": " << step << ", \"t\": " << step * p.tau
    << ", \"shape\": [" << l.nx << ", " << l.ny << ", " << l.nz << "], \"offset\": [" << l.gx0 << ", " << l.gy0
    << ", " << l.gz0 << "], \"global_shape\": [" << p.N + 1 << ", " << p.N + 1 << ", " << p.N + 1
    << "], \"rank\": " << rank << ", \"world\": " << world << ", \"dims\": [" << d.px << ", " << d.py << ", " << d.pz
    << "]}\n";
}

// --checkpoint PREFIX: u^K → PREFIX.cur, u^{K−1} → PREFIX.prev (wave3d-dump-v1, per rank when world > 1)
void write_checkpoint(const std::string& prefix, const Problem& p, const Layout& l, const std::vector<double>& cur,
                      const std::vector<double>& prev, int rank, int world, const Dims& d) {
  write_dump(prefix + ".cur", p, l, cur, rank, world, d, p.K);
  write_dump(prefix + ".prev", p, l, prev, rank, world, d, p.K - 1);
}

// Number after "key": in a one-line JSON object (the dump sidecars this program writes).
std::vector<double> json_numbers(const std::string& text, const std::string& key) {
  std::vector<double> out;
  const size_t k = text.find("\"" + key + "\"");
  if (k == std::string::npos) return out;
  size_t i = text.find(':', k) + 1;
  const bool list = text.find_first_not_of(" ", i) != std::string::npos && text[text.find_first_not_of(" ", i)] == '[';
  if (list) i = text.find('[', i) + 1;
  for (;;) {
    char* end = nullptr;
    const double v = std::strtod(text.c_str() + i, &end);
    if (end == text.c_str() + i) break;
    out.push_back(v);
    i = static_cast<size_t>(end - text.c_str());
    if (!list) break;
    i = text.find_first_of(",]", i);
    if (i == std::string::npos || text[i] == ']') break;
    ++i;
  }
  return out;
}

// The GLOBAL (N+1)³ field of a dump PREFIX (one file, or PREFIX.rankR of any decomposition); returns its step.
int load_dump_global(const std::string& prefix, const Problem& p, std::vector<double>& g) {
  auto slurp = [](const std::string& path) {
    std::ifstream f(path);
    return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  };
  std::string meta = slurp(prefix + ".json");
  std::vector<std::string> bases;
  if (!meta.empty()) {
    bases.push_back(prefix);
  } else {
    meta = slurp(prefix + ".rank0.json");
    W3D_REQUIRE(!meta.empty(), "resume: no dump " + prefix + ".json or " + prefix + ".rank0.json");
    const std::vector<double> w = json_numbers(meta, "world");
    W3D_REQUIRE(!w.empty() && w[0] >= 1, "resume: dump without a world size");
    for (int r = 0; r < static_cast<int>(w[0]); ++r) bases.push_back(prefix + ".rank" + std::to_string(r));
  }
  const i64 n1 = p.N + 1;
  g.assign(static_cast<size_t>(n1 * n1 * n1), 0.0);
  int step = -1;
  for (const std::string& b : bases) {
    const std::string m = slurp(b + ".json");
    const std::vector<double> sh = json_numbers(m, "shape"), of = json_numbers(m, "offset"), st = json_numbers(m, "step"),
                              nn = json_numbers(m, "N");
    W3D_REQUIRE(sh.size() == 3 && of.size() == 3 && st.size() == 1 && nn.size() == 1, "resume: bad sidecar " + b);
    W3D_REQUIRE(static_cast<i64>(nn[0]) == p.N, "resume: dump N differs from the run's N");
    // (tau and L too: a checkpoint of another problem would continue from an inconsistent state; the sidecar holds
    // them with 17 significant digits, so they round-trip exactly)
    for (const auto& [key, want] : {std::pair<const char*, double>{"tau", p.tau}, {"L", p.L}}) {
      const std::vector<double> v = json_numbers(m, key);
      W3D_REQUIRE(v.size() == 1 && std::fabs(v[0] - want) <= 1e-15 * std::fabs(want),
                  std::string("resume: dump ") + key + " differs from the run's " + key);
    }
    W3D_REQUIRE(step < 0 || step == static_cast<int>(st[0]), "resume: rank dumps of different steps");
    step = static_cast<int>(st[0]);
    const i64 nx = static_cast<i64>(sh[0]), ny = static_cast<i64>(sh[1]), nz = static_cast<i64>(sh[2]);
    const i64 x0 = static_cast<i64>(of[0]), y0 = static_cast<i64>(of[1]), z0 = static_cast<i64>(of[2]);
    W3D_REQUIRE(x0 >= 0 && y0 >= 0 && z0 >= 0 && x0 + nx <= n1 && y0 + ny <= n1 && z0 + nz <= n1,
                "resume: dump box outside the grid");
    std::ifstream f(b + ".bin", std::ios::binary);
    W3D_REQUIRE(static_cast<bool>(f), "resume: cannot read " + b + ".bin");
    for (i64 x = 0; x < nx; ++x)
      for (i64 y = 0; y < ny; ++y)
        f.read(reinterpret_cast<char*>(g.data() + ((x0 + x) * n1 + (y0 + y)) * n1 + z0),
               static_cast<std::streamsize>(nz * static_cast<i64>(sizeof(double))));
    W3D_REQUIRE(static_cast<bool>(f), "resume: short file " + b + ".bin");
  }
  return step;
}

// --resume PREFIX: u^{n0−1} from PREFIX.prev, u^{n0} from PREFIX.cur; returns n0
int load_checkpoint(const std::string& prefix, const Problem& p, std::vector<double>& prev, std::vector<double>& cur) {
  const int sc = load_dump_global(prefix + ".cur", p, cur);
  const int sp = load_dump_global(prefix + ".prev", p, prev);
  W3D_REQUIRE(sp == sc - 1, "resume: PREFIX.prev must hold the step before PREFIX.cur");
  W3D_REQUIRE(sc >= 1 && sc < p.K, "resume: checkpoint step " + std::to_string(sc) + " is not before K");
  return sc;
}

}  // namespace wave3d
