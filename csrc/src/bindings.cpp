// Python bindings of the native runtime (pybind11). Module: mpi_cuda_amd._C
//
// The GPU path is fully native (GpuSolver: HIP kernels + RCCL, C++ step loop, hipGraph). The raw kernel launchers take
// device pointers as integers (torch.Tensor.data_ptr()) and a stream handle (torch.cuda.current_stream().cuda_stream)
// so the tests can drive each kernel against a PyTorch fp64 reference. The CPU kernels take numpy float64 arrays.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "wave3d/capture_guard.hpp"
#include "wave3d/cpu.hpp"
#include "wave3d/decomp.hpp"
#include "wave3d/kernels.hpp"
#include "wave3d/problem.hpp"
#include "wave3d/runtime.hpp"
#include "wave3d/solver.hpp"
#include "wave3d/stencil.hpp"

namespace py = pybind11;
using namespace wave3d;

namespace {

using darr = py::array_t<double, py::array::c_style | py::array::forcecast>;

double* mut_ptr(darr& a, i64 need, const char* what) {
  W3D_REQUIRE(a.size() >= need, std::string(what) + ": array too small");
  return a.mutable_data();
}
const double* ro_ptr(const darr& a, i64 need, const char* what) {
  W3D_REQUIRE(a.size() >= need, std::string(what) + ": array too small");
  return a.data();
}

template <class T>
T* dptr(std::uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
hipStream_t sptr(std::uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

py::dict result_dict(const RunResult& r) {
  py::dict d;
  d["steps"] = r.steps;
  d["max_err"] = r.max_err;
  d["rms_err"] = r.rms_err;
  d["solve_s"] = r.solve_s;
  d["batched"] = r.batched;
  d["finite"] = r.finite;
  py::dict ph;
  ph["init_ms"] = r.phases.init_ms;
  ph["shell_ms"] = r.phases.shell_ms;
  ph["compute_ms"] = r.phases.interior_ms;
  ph["comm_ms"] = r.phases.comm_ms;
  ph["check_ms"] = r.phases.check_ms;
  ph["gather_ms"] = r.phases.gather_ms;
  d["phases"] = ph;
  py::list tr;
  for (const UnitTrace& t : r.trace) {
    py::dict u;
    u["unit"] = t.unit;
    u["n"] = t.n;
    u["steps"] = t.steps;
    u["shell_ms"] = t.shell_ms;
    u["comm_ms"] = t.comm_ms;
    u["compute_ms"] = t.compute_ms;
    u["check_ms"] = t.check_ms;
    tr.append(u);
  }
  d["trace"] = tr;
  return d;
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "wave3d native runtime: CDNA4 HIP kernels, RCCL halo exchange, CPU/OpenMP path";

  py::class_<Problem>(m, "Problem")
      .def(py::init([](i64 N, double tau, int K, double L) {
             Problem p;
             p.N = N;
             p.tau = tau;
             p.K = K;
             p.L = L;
             p.validate();
             return p;
           }),
           py::arg("N") = 512, py::arg("tau") = 1e-3, py::arg("K") = 20, py::arg("L") = 1.0)
      .def_readwrite("N", &Problem::N)
      .def_readwrite("tau", &Problem::tau)
      .def_readwrite("K", &Problem::K)
      .def_readwrite("L", &Problem::L)
      .def_property_readonly("h", &Problem::h)
      .def_property_readonly("a_t", &Problem::a_t)
      .def_property_readonly("courant", &Problem::courant)
      .def_property_readonly("cfl_ok", &Problem::cfl_ok)
      .def_property_readonly("tau_max", &Problem::tau_max)
      .def_property_readonly("cell_updates", &Problem::cell_updates)
      .def("__repr__", [](const Problem& p) {
        return "Problem(N=" + std::to_string(p.N) + ", tau=" + std::to_string(p.tau) + ", K=" + std::to_string(p.K) +
               ", L=" + std::to_string(p.L) + ")";
      });

  py::class_<Coeffs>(m, "Coeffs")
      .def_static("from_problem", &Coeffs::from)
      .def_readonly("ihx2", &Coeffs::ihx2)
      .def_readonly("ihy2", &Coeffs::ihy2)
      .def_readonly("ihz2", &Coeffs::ihz2)
      .def_readonly("tau2", &Coeffs::tau2)
      .def_readonly("half_tau2", &Coeffs::half_tau2)
      .def_readonly("lam", &Coeffs::lam)
      .def_readonly("half_lam", &Coeffs::half_lam);

  m.def("sin_table_ext", [](const Problem& p) {
    auto v = sin_table_ext(p);
    return darr(static_cast<py::ssize_t>(v.size()), v.data());
  });
  m.def("time_factor", &time_factor);
  // elementwise IEEE fused multiply-add (the rounding of stencil.hpp's leapfrog / first_step / err_sq_acc), for the
  // numpy emulators that must reproduce the kernels bit for bit (numpy has no fma)
  m.def("fma_array", [](const darr& a, const darr& b, const darr& c) {
    W3D_REQUIRE(a.size() == b.size() && a.size() == c.size(), "fma_array: sizes differ");
    darr out(a.size());
    double* o = out.mutable_data();
    const double *pa = a.data(), *pb = b.data(), *pc = c.data();
    for (py::ssize_t i = 0; i < a.size(); ++i) o[i] = fma_exact(pa[i], pb[i], pc[i]);
    return out;
  });

  py::class_<Dims>(m, "Dims")
      .def(py::init([](int px, int py_, int pz) { return Dims{px, py_, pz}; }))
      .def_readwrite("px", &Dims::px)
      .def_readwrite("py", &Dims::py)
      .def_readwrite("pz", &Dims::pz)
      .def("size", &Dims::size)
      .def("as_tuple", [](const Dims& d) { return py::make_tuple(d.px, d.py, d.pz); });
  m.def("parse_dims", &parse_dims);
  m.def("block_dims", &block_dims);
  m.def("split_axis", [](i64 N, int p, int c) {
    i64 b, e;
    split_axis(N, p, c, &b, &e);
    return py::make_tuple(b, e);
  });

  py::class_<Box>(m, "Box")
      .def_readonly("x0", &Box::x0)
      .def_readonly("x1", &Box::x1)
      .def_readonly("y0", &Box::y0)
      .def_readonly("y1", &Box::y1)
      .def_readonly("z0", &Box::z0)
      .def_readonly("z1", &Box::z1)
      .def("count", &Box::count);
  m.def("rank_box", &rank_box);
  m.def("neighbor_rank", &neighbor_rank);
  m.def("rank_coords", &rank_coords);

  py::class_<Layout>(m, "Layout")
      .def_readonly("N", &Layout::N)
      .def_readonly("xg", &Layout::xg)
      .def_readonly("yg", &Layout::yg)
      .def_readonly("zg", &Layout::zg)
      .def("zero_off", &Layout::zero_off)
      .def_readonly("nx", &Layout::nx)
      .def_readonly("ny", &Layout::ny)
      .def_readonly("nz", &Layout::nz)
      .def_readonly("gx0", &Layout::gx0)
      .def_readonly("gy0", &Layout::gy0)
      .def_readonly("gz0", &Layout::gz0)
      .def_readonly("zs", &Layout::zs)
      .def_readonly("pitch", &Layout::pitch)
      .def_readonly("plane", &Layout::plane)
      .def_readonly("total", &Layout::total)
      .def_readonly("cx0", &Layout::cx0)
      .def_readonly("cx1", &Layout::cx1)
      .def_readonly("cy0", &Layout::cy0)
      .def_readonly("cy1", &Layout::cy1)
      .def_readonly("cz0", &Layout::cz0)
      .def_readonly("cz1", &Layout::cz1)
      .def("off", [](const Layout& l, i64 x, i64 y, i64 z) { return l.off(x, y, z); });
  m.def("make_layout", &make_layout, py::arg("problem"), py::arg("box"), py::arg("pitch_align") = 16,
        py::arg("xg") = 1, py::arg("yg") = 1, py::arg("zg") = 1);

  py::class_<Face>(m, "Face")
      .def_readonly("axis", &Face::axis)
      .def_readonly("side", &Face::side)
      .def_readonly("peer", &Face::peer)
      .def_readonly("count", &Face::count)
      .def_readonly("contiguous", &Face::contiguous)
      .def_readonly("send_off", &Face::send_off)
      .def_readonly("recv_off", &Face::recv_off)
      .def_readonly("send_layer", &Face::send_layer)
      .def_readonly("recv_layer", &Face::recv_layer)
      .def_readonly("pack_off", &Face::pack_off);
  py::class_<HaloPlan>(m, "HaloPlan")
      .def_readonly("faces", &HaloPlan::faces)
      .def_readonly("packed_doubles", &HaloPlan::packed_doubles);
  m.def("make_halo_plan", &make_halo_plan);

  py::class_<DeepPart>(m, "DeepPart")
      .def_readonly("field", &DeepPart::field)
      .def_readonly("send", &DeepPart::send)
      .def_readonly("recv", &DeepPart::recv)
      .def_readonly("off", &DeepPart::off);
  py::class_<DeepPeer>(m, "DeepPeer")
      .def_readonly("peer", &DeepPeer::peer)
      .def_readonly("dir", &DeepPeer::dir)
      .def_readonly("count", &DeepPeer::count)
      .def_readonly("buf_off", &DeepPeer::buf_off)
      .def_readonly("parts", &DeepPeer::parts);
  py::class_<DeepPlan>(m, "DeepPlan")
      .def_readonly("s", &DeepPlan::s)
      .def_readonly("peers", &DeepPlan::peers)
      .def_readonly("total", &DeepPlan::total);
  m.def("make_deep_plan", &make_deep_plan, py::arg("layout"), py::arg("dims"), py::arg("rank"), py::arg("s"));

  py::class_<LBox>(m, "LBox")
      .def(py::init([](i64 x0, i64 x1, i64 y0, i64 y1, i64 z0, i64 z1) { return LBox{x0, x1, y0, y1, z0, z1}; }))
      .def_readwrite("x0", &LBox::x0)
      .def_readwrite("x1", &LBox::x1)
      .def_readwrite("y0", &LBox::y0)
      .def_readwrite("y1", &LBox::y1)
      .def_readwrite("z0", &LBox::z0)
      .def_readwrite("z1", &LBox::z1)
      .def("empty", &LBox::empty)
      .def("count", &LBox::count)
      .def("as_tuple", [](const LBox& b) { return py::make_tuple(b.x0, b.x1, b.y0, b.y1, b.z0, b.z1); });
  m.def("compute_box", &compute_box);
  m.def(
      "shell_split",
      [](const LBox& full, const std::vector<std::vector<bool>>& nbv) {
        W3D_REQUIRE(nbv.size() == 3 && nbv[0].size() == 2 && nbv[1].size() == 2 && nbv[2].size() == 2,
                    "shell_split: neighbours as [[x lo, x hi], [y lo, y hi], [z lo, z hi]]");
        bool nb[3][2];
        for (int a = 0; a < 3; ++a)
          for (int s = 0; s < 2; ++s) nb[a][s] = nbv[static_cast<size_t>(a)][static_cast<size_t>(s)];
        std::vector<LBox> shell;
        LBox interior;
        shell_split(full, nb, shell, interior);
        return py::make_tuple(shell, interior);
      },
      "(shell boxes, interior box) of a compute box with neighbours nb[axis][side] (the runtime's own split)");
  m.def(
      "deep_split",
      [](const LBox& full, const std::vector<std::vector<bool>>& nbv, i64 w, i64 tile) {
        W3D_REQUIRE(nbv.size() == 3 && nbv[0].size() == 2 && nbv[1].size() == 2 && nbv[2].size() == 2,
                    "deep_split: neighbours as [[x lo, x hi], [y lo, y hi], [z lo, z hi]]");
        bool nb[3][2];
        for (int a = 0; a < 3; ++a)
          for (int s = 0; s < 2; ++s) nb[a][s] = nbv[static_cast<size_t>(a)][static_cast<size_t>(s)];
        std::vector<LBox> shell;
        LBox interior;
        deep_split(full, nb, w, tile, shell, interior);
        return py::make_tuple(shell, interior);
      },
      py::arg("full"), py::arg("nb"), py::arg("w"), py::arg("tile") = 32,
      "(shell boxes, interior box) of a deep-tb unit whose exchange of depth w overlaps the pass (GpuSolver::tb_split)");

  // ---------------- CPU kernels ----------------
  m.def("cpu_set_threads", &cpu_set_threads);
  m.def("cpu_max_threads", &cpu_max_threads);
  m.def("cpu_init_first", [](const Layout& l, const Coeffs& c, const darr& s, darr u0, darr u1) {
    const double* sp = ro_ptr(s, l.N + 3, "s") + 1;
    double* a = mut_ptr(u0, l.total, "u0");
    double* b = mut_ptr(u1, l.total, "u1");
    py::gil_scoped_release nogil;
    cpu_init_first(l, c, sp, a, b);
  });
  m.def(
      "cpu_leapfrog",
      [](const Layout& l, const Coeffs& c, const darr& cur, darr old, const LBox& box, const darr& s, double ct,
         bool check) -> py::object {
        const double* cp = ro_ptr(cur, l.total, "cur");
        double* op = mut_ptr(old, l.total, "old");
        const double* sp = ro_ptr(s, l.N + 3, "s") + 1;
        ErrAcc acc;
        {
          py::gil_scoped_release nogil;
          cpu_leapfrog(l, c, cp, op, box, sp, ct, check ? &acc : nullptr);
        }
        if (!check) return py::none();
        return py::make_tuple(acc.max, acc.sum);
      },
      py::arg("layout"), py::arg("coeffs"), py::arg("cur"), py::arg("old"), py::arg("box"), py::arg("s"),
      py::arg("ct") = 0.0, py::arg("check") = false);
  m.def("cpu_error", [](const Layout& l, const darr& u, const LBox& box, const darr& s, double ct) {
    ErrAcc acc;
    cpu_error(l, ro_ptr(u, l.total, "u"), box, ro_ptr(s, l.N + 3, "s") + 1, ct, &acc);
    return py::make_tuple(acc.max, acc.sum);
  });
  m.def("cpu_pack_face", [](const Layout& l, const Face& f, const darr& u, darr buf) {
    cpu_pack_face(l, f, ro_ptr(u, l.total, "u"), mut_ptr(buf, f.count, "buf"));
  });
  m.def("cpu_unpack_face", [](const Layout& l, const Face& f, const darr& buf, darr u) {
    cpu_unpack_face(l, f, ro_ptr(buf, f.count, "buf"), mut_ptr(u, l.total, "u"));
  });

  py::class_<CpuSolver>(m, "CpuSolver")
      .def(py::init<const Problem&, int, int>(), py::arg("problem"), py::arg("check_every") = 2,
           py::arg("threads") = 0)
      .def("run",
           [](CpuSolver& s) {
             CpuResult r;
             {
               py::gil_scoped_release nogil;
               r = s.run();
             }
             py::dict d;
             d["steps"] = r.steps;
             d["max_err"] = r.max_err;
             d["rms_err"] = r.rms_err;
             d["solve_s"] = r.solve_s;
             d["init_s"] = r.init_s;
             d["compute_s"] = r.compute_s;
             d["finite"] = r.finite;
             return d;
           })
      .def("field",
           [](const CpuSolver& s, int which) {
             const auto& v = s.field(which);
             return darr(static_cast<py::ssize_t>(v.size()), v.data());
           })
      .def_property_readonly("layout", &CpuSolver::layout)
      .def("check_steps", &CpuSolver::check_steps)
      .def("set_state", [](CpuSolver& s, const darr& prev, const darr& cur, int n0) {
        const i64 n = s.layout().N + 1;
        s.set_state(ro_ptr(prev, n * n * n, "prev"), ro_ptr(cur, n * n * n, "cur"), n0);
      }, py::arg("prev"), py::arg("cur"), py::arg("step"));

  // ---------------- GPU ----------------
  m.def("gpu_device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return n;
  });
  m.def("gpu_set_device", [](int d) { W3D_HIP(hipSetDevice(d)); });
  // versions of the HIP runtime and RCCL this process actually resolved (torch may have loaded its bundled copies)
  m.def("runtime_versions", []() {
    int hv = 0, dv = 0, nv = 0;
    (void)hipRuntimeGetVersion(&hv);
    (void)hipDriverGetVersion(&dv);
    nv = rccl_version();
    py::dict d;
    d["hip_runtime"] = hv;
    d["hip_driver"] = dv;
    d["rccl"] = nv;
    d["multistream_capture_safe"] = multistream_capture_safe();
    return d;
  });
  m.def("gpu_synchronize", []() { W3D_HIP(hipDeviceSynchronize()); });
  m.def("gpu_arch", []() {
    int d = 0;
    W3D_HIP(hipGetDevice(&d));
    hipDeviceProp_t p;
    W3D_HIP(hipGetDeviceProperties(&p, d));
    return std::string(p.gcnArchName);
  });

  py::class_<LeapfrogTiling>(m, "LeapfrogTiling")
      .def(py::init<>())
      .def_readwrite("variant", &LeapfrogTiling::variant)
      .def_readwrite("rows", &LeapfrogTiling::rows)
      .def_readwrite("ty", &LeapfrogTiling::ty)
      .def_readwrite("target_blocks", &LeapfrogTiling::target_blocks)
      .def_readwrite("xcd_remap", &LeapfrogTiling::xcd_remap)
      .def_readwrite("nt_store", &LeapfrogTiling::nt_store);

  m.def("gpu_init_first", [](const Layout& l, const Coeffs& c, std::uintptr_t s, std::uintptr_t u0, std::uintptr_t u1,
                             std::uintptr_t stream) {
    launch_init_first(l, c, dptr<const double>(s) + 1, dptr<double>(u0), dptr<double>(u1), sptr(stream));
  });
  m.def("gpu_init_two_partials", &init_two_partials);
  m.def("gpu_init_two", [](const Layout& l, const Coeffs& c, std::uintptr_t s, std::uintptr_t u1, std::uintptr_t u2,
                           double ct2, std::uintptr_t partials, std::uintptr_t stream) {
    launch_init_two(l, c, dptr<const double>(s) + 1, dptr<double>(u1), dptr<double>(u2), ct2,
                    dptr<Partial>(partials), sptr(stream));
  });
  m.def("gpu_leapfrog_blocks", [](const Layout& l, const std::vector<LBox>& boxes, const LeapfrogTiling& t) {
    return leapfrog_blocks(l, boxes.data(), static_cast<int>(boxes.size()), t);
  });
  m.def("gpu_leapfrog",
        [](const Layout& l, const Coeffs& c, std::uintptr_t cur, std::uintptr_t old, const std::vector<LBox>& boxes,
           std::uintptr_t s, double ct, std::uintptr_t partials, const LeapfrogTiling& t, std::uintptr_t stream) {
          launch_leapfrog(l, c, dptr<const double>(cur), dptr<double>(old), boxes.data(),
                          static_cast<int>(boxes.size()), dptr<const double>(s) + 1, ct, dptr<Partial>(partials), t,
                          sptr(stream));
        });
  py::class_<Leapfrog2Tiling>(m, "Leapfrog2Tiling")
      .def(py::init<>())
      .def_readwrite("rows", &Leapfrog2Tiling::rows)
      .def_readwrite("target_waves", &Leapfrog2Tiling::target_waves)
      .def_readwrite("occupancy", &Leapfrog2Tiling::occupancy)
      .def_readwrite("xcd_remap", &Leapfrog2Tiling::xcd_remap)
      .def_readwrite("nt_store", &Leapfrog2Tiling::nt_store);
  m.def("gpu_leapfrog2_partials", &leapfrog2_partials);
  m.def("gpu_leapfrog2",
        [](const Layout& l, const Coeffs& c, std::uintptr_t prev, std::uintptr_t cur, std::uintptr_t out1,
           std::uintptr_t out2, const LBox& box, std::uintptr_t s, double ct2, std::uintptr_t partials,
           const Leapfrog2Tiling& t, std::uintptr_t stream, i64 sx0, i64 sx1) {
          launch_leapfrog2(l, c, dptr<const double>(prev), dptr<const double>(cur), dptr<double>(out1),
                           dptr<double>(out2), box, dptr<const double>(s) + 1, ct2, dptr<Partial>(partials), t,
                           sptr(stream), sx0, sx1);
        },
        py::arg("layout"), py::arg("coeffs"), py::arg("prev"), py::arg("cur"), py::arg("out1"), py::arg("out2"),
        py::arg("box"), py::arg("s"), py::arg("ct2"), py::arg("partials"), py::arg("tiling"), py::arg("stream"),
        py::arg("sx0") = 1, py::arg("sx1") = 0);
  py::class_<LeapfrogTbTiling>(m, "LeapfrogTbTiling")
      .def(py::init<>())
      .def_readwrite("stages", &LeapfrogTbTiling::stages)
      .def_readwrite("threads", &LeapfrogTbTiling::threads)
      .def_readwrite("init_threads", &LeapfrogTbTiling::init_threads)
      .def_readwrite("xcd_remap", &LeapfrogTbTiling::xcd_remap)
      .def_readwrite("xcd_blocks", &LeapfrogTbTiling::xcd_blocks)
      .def_readwrite("target_blocks", &LeapfrogTbTiling::target_blocks)
      .def_readwrite("min_chunk", &LeapfrogTbTiling::min_chunk)
      .def_readwrite("p2", &LeapfrogTbTiling::p2)
      .def_readwrite("ghost_x1", &LeapfrogTbTiling::ghost_x1);
  m.def("capture_guard_selftest", &wave3d::capture::selftest, py::arg("mode"),
        "the probe topologies through the stream-capture guard (0: production, 2: the round-4 sibling wait)");
  m.def("leapfrog_p2_table", [](int stages) {
        std::vector<long> geo;
        std::vector<int> t = wave3d::leapfrog_p2_table(stages, &geo);
        return py::make_tuple(t, geo);
      }, py::arg("stages"), "the pair-tiled pass's compile-time thread table and geometry (host copy, no GPU)");
  m.def("gpu_leapfrog_p2_supported", &leapfrog_p2_supported);
  m.def("gpu_leapfrog_tb_lds_bytes", &leapfrog_tb_lds_bytes);
  m.def("gpu_leapfrog_tb_partials", &leapfrog_tb_partials);
  m.def("gpu_leapfrog_tb",
        [](const Layout& l, const Coeffs& c, std::uintptr_t prev, std::uintptr_t cur, std::uintptr_t out1,
           std::uintptr_t out2, const LBox& box, std::uintptr_t s, std::vector<double> ct, int check_mask,
           std::uintptr_t partials, const LeapfrogTbTiling& t, std::uintptr_t stream, const LBox& real,
           bool analytic_start) {
          ct.resize(5, 0.0);
          launch_leapfrog_tb(l, c, dptr<const double>(prev), dptr<const double>(cur), dptr<double>(out1),
                             dptr<double>(out2), box, dptr<const double>(s) + 1, ct.data(), check_mask,
                             dptr<Partial>(partials), t, sptr(stream), real, analytic_start);
        },
        py::arg("layout"), py::arg("coeffs"), py::arg("prev"), py::arg("cur"), py::arg("out1"), py::arg("out2"),
        py::arg("box"), py::arg("s"), py::arg("ct"), py::arg("check_mask"), py::arg("partials"), py::arg("tiling"),
        py::arg("stream"), py::arg("real") = tb_default_real(), py::arg("analytic_start") = false);
  m.def("gpu_error_blocks", &error_blocks);
  m.def("gpu_error", [](const Layout& l, std::uintptr_t u, const LBox& b, std::uintptr_t s, double ct,
                        std::uintptr_t partials, std::uintptr_t stream) {
    launch_error(l, dptr<const double>(u), b, dptr<const double>(s) + 1, ct, dptr<Partial>(partials), sptr(stream));
  });
  m.def("gpu_reduce_batch", [](const std::vector<std::tuple<std::uintptr_t, int, std::uintptr_t>>& jobs,
                               std::uintptr_t stream) {
    std::vector<ReduceJob> js;
    for (const auto& [in, n, out] : jobs) js.push_back(ReduceJob{dptr<const Partial>(in), n, dptr<Partial>(out)});
    launch_reduce_batch(js.data(), static_cast<int>(js.size()), sptr(stream));
  });
  m.def("gpu_reduce", [](std::uintptr_t partials, int n, std::uintptr_t out, std::uintptr_t stream) {
    launch_reduce(dptr<const Partial>(partials), n, dptr<Partial>(out), sptr(stream));
  });
  m.def("gpu_pack", [](const Layout& l, const HaloPlan& p, std::uintptr_t u, std::uintptr_t buf, std::uintptr_t st) {
    launch_pack(l, p, dptr<const double>(u), dptr<double>(buf), sptr(st));
  });
  m.def("gpu_unpack", [](const Layout& l, const HaloPlan& p, std::uintptr_t buf, std::uintptr_t u, std::uintptr_t st) {
    launch_unpack(l, p, dptr<const double>(buf), dptr<double>(u), sptr(st));
  });

  py::class_<SolverOptions>(m, "SolverOptions")
      .def(py::init<>())
      .def_readwrite("decomp", &SolverOptions::decomp)
      .def_readwrite("check_every", &SolverOptions::check_every)
      .def_readwrite("overlap", &SolverOptions::overlap)
      .def_readwrite("graph", &SolverOptions::graph)
      .def_readwrite("timers", &SolverOptions::timers)
      .def_readwrite("debug_sync", &SolverOptions::debug_sync)
      .def_readwrite("poison_ghosts", &SolverOptions::poison_ghosts)
      .def_readwrite("fake_comm", &SolverOptions::fake_comm)
      .def_readwrite("push", &SolverOptions::push)
      .def_readwrite("push_cp_wait", &SolverOptions::push_cp_wait)
      .def_readwrite("sdma", &SolverOptions::sdma)
      .def_readwrite("shells_concurrent", &SolverOptions::shells_concurrent)
      .def_readwrite("reserve_cus", &SolverOptions::reserve_cus)
      .def_readwrite("fake_traffic", &SolverOptions::fake_traffic)
      .def_readwrite("fused_pack", &SolverOptions::fused_pack)
      .def_readwrite("ghost_store", &SolverOptions::ghost_store)
      .def_readwrite("sdma_streams", &SolverOptions::sdma_streams)
      .def_readwrite("flag_timeout_s", &SolverOptions::flag_timeout_s)
      .def_readwrite("push_no_collective", &SolverOptions::push_no_collective)
      .def_readwrite("temporal", &SolverOptions::temporal)
      .def_readwrite("init2", &SolverOptions::init2)
      .def_readwrite("deep_min_planes", &SolverOptions::deep_min_planes)
      .def_readwrite("tb_min_planes", &SolverOptions::tb_min_planes)
      .def_readwrite("tiling2", &SolverOptions::tiling2)
      .def_readwrite("tb", &SolverOptions::tb)
      .def_readwrite("tiling_tb", &SolverOptions::tiling_tb)
      .def_readwrite("tiling", &SolverOptions::tiling);

  py::class_<Comm, std::shared_ptr<Comm>>(m, "Comm")
      .def(py::init([](int rank, int world, py::bytes uid) {
             std::string s = uid;
             py::gil_scoped_release nogil;
             return std::make_shared<Comm>(rank, world, s);
           }),
           py::arg("rank"), py::arg("world"), py::arg("unique_id"))
      .def_static("make_unique_id", []() { return py::bytes(Comm::make_unique_id()); })
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("world", &Comm::world)
      .def("count", &Comm::count)
      .def("device", &Comm::device)
      .def("check_async", &Comm::check_async);

  py::class_<GpuSolver>(m, "GpuSolver")
      .def(py::init([](const Problem& p, const SolverOptions& o, int rank, int world, std::shared_ptr<Comm> c) {
             return std::make_unique<GpuSolver>(p, o, rank, world, std::move(c));
           }),
           py::arg("problem"), py::arg("options"), py::arg("rank") = 0, py::arg("world") = 1,
           py::arg("comm") = nullptr)
      .def_property_readonly("push", &GpuSolver::push)
      .def("push_handles", [](const GpuSolver& s) { return py::bytes(s.push_handles()); },
           "this rank's IPC handles (staging, flags) + device, to be all-gathered")
      .def("connect_push", [](GpuSolver& s, const std::vector<py::bytes>& all) {
             std::vector<std::string> v;
             for (const py::bytes& b : all) v.emplace_back(b);
             s.connect_push(v);
           },
           "open the slab neighbours' staging and flags from every rank's push_handles() (index = rank)")
      .def_property_readonly("sdma", &GpuSolver::sdma)
      .def("sdma_handles", [](const GpuSolver& s) { return py::bytes(s.sdma_handles()); },
           "this rank's IPC handles (field buffers, staging, flags) + layout facts, to be all-gathered")
      .def("connect_sdma", [](GpuSolver& s, const std::vector<py::bytes>& all) {
             std::vector<std::string> v;
             for (const py::bytes& b : all) v.emplace_back(b);
             s.connect_sdma(v);
           },
           "map every neighbour's buffers and flag words from all ranks' sdma_handles() (index = rank)")
      .def_property_readonly("overlapped", &GpuSolver::overlapped)
      .def_property_readonly("transport", &GpuSolver::transport)
      .def("traffic",
           [](GpuSolver& s) {
             const GpuSolver::Traffic t = s.traffic();
             py::dict d;
             d["field_bytes"] = t.field_bytes;
             d["halo_bytes"] = t.halo_bytes;
             return d;
           },
           "bytes one solve of the last run()'s schedule moves: compulsory field reads + writes, halo bytes sent")
      .def("run",
           [](GpuSolver& s) {
             RunResult r;
             {
               py::gil_scoped_release nogil;
               r = s.run();
             }
             return result_dict(r);
           })
      .def("run_batch",
           [](GpuSolver& s, int n) {
             std::vector<RunResult> rs;
             {
               py::gil_scoped_release nogil;
               rs = s.run_batch(n);
             }
             py::list out;
             for (const RunResult& r : rs) out.append(result_dict(r));
             return out;
           },
           py::arg("n"),
           "n solves back to back; a one-rank graph-captured solver enqueues them all and synchronises once (each "
           "solve's own log copied out)")
      .def("download",
           [](const GpuSolver& s, int which) {
             auto v = s.download(which);
             return darr(static_cast<py::ssize_t>(v.size()), v.data());
           },
           py::arg("which") = 0)
      .def("field_hash", &GpuSolver::field_hash, py::arg("which") = 0,
           "order-independent 64-bit hash of the owned nodes of u^K (0) / u^{K-1} (1); summed over the ranks it is "
           "the same for every decomposition that computes bit-identical fields")
      .def_property_readonly("layout", &GpuSolver::layout)
      .def_property_readonly("dims", &GpuSolver::dims)
      .def_property_readonly("halo", &GpuSolver::halo)
      .def_property_readonly("rank", &GpuSolver::rank)
      .def_property_readonly("world", &GpuSolver::world)
      .def("set_state", [](GpuSolver& s, const darr& prev, const darr& cur, int n0) {
        const i64 n = s.problem().N + 1;
        s.set_state(ro_ptr(prev, n * n * n, "prev"), ro_ptr(cur, n * n * n, "cur"), n0);
      }, py::arg("prev"), py::arg("cur"), py::arg("step"))
      .def("shell_boxes", &GpuSolver::shell_boxes)
      .def("interior_box", &GpuSolver::interior_box)
      .def("check_steps", &GpuSolver::check_steps)
      .def("device_bytes", &GpuSolver::device_bytes)
      .def_property_readonly("mode", &GpuSolver::mode)
      .def_property_readonly("graph_enabled", [](const GpuSolver& s) { return s.options().graph; });

  // the CLI's multi-rank schedule autotune (runtime_autotune.cpp): same candidates, same rules; collectives over the
  // RCCL communicator (world > 1) or none (one rank / a fake rank)
  m.def(
      "autotune",
      [](const Problem& p, const SolverOptions& o, int rank, int world, std::shared_ptr<Comm> c, bool fake,
         bool with_push, int rounds, double tie, bool with_sdma, int reps, double budget_s) {
        W3D_REQUIRE(world == 1 || fake || c, "autotune: world > 1 needs an RCCL communicator");
        const HostColl hc = c ? HostColl::rccl(c) : HostColl::single(rank);
        AutotuneOptions ao;
        ao.with_push = with_push;
        ao.with_sdma = with_sdma;
        ao.rounds = rounds;
        ao.reps = reps;
        ao.tie = tie;
        ao.budget_s = budget_s;
        AutotuneResult r;
        {
          py::gil_scoped_release nogil;
          r = autotune(p, o, rank, world, c, hc, fake, ao);
        }
        py::dict times, rejected;
        for (const auto& [k, v] : r.times) times[py::str(k)] = v;
        for (const auto& [k, v] : r.rejected) rejected[py::str(k)] = v;
        return py::make_tuple(py::cast(std::move(r.solver)), r.name, times, rejected);
      },
      py::arg("problem"), py::arg("options"), py::arg("rank") = 0, py::arg("world") = 1, py::arg("comm") = nullptr,
      py::arg("fake") = false, py::arg("with_push") = false, py::arg("rounds") = 5, py::arg("tie") = 0.02,
      py::arg("with_sdma") = false, py::arg("reps") = 5, py::arg("budget_s") = 120.0,
      "time the schedule candidates (slab/block, pass depth, overlap, RCCL/copy engines) and return "
      "(GpuSolver, name, {name: seconds}, {name: reason rejected})");

  py::class_<GpuGroup>(m, "GpuGroup")
      .def(py::init([](const Problem& p, const SolverOptions& o, int world, const std::string& transport) {
             py::gil_scoped_release nogil;
             return std::make_unique<GpuGroup>(p, o, world, transport);
           }),
           py::arg("problem"), py::arg("options"), py::arg("world"), py::arg("transport") = "loopback")
      .def("run",
           [](GpuGroup& g) {
             RunResult r;
             {
               py::gil_scoped_release nogil;
               r = g.run();
             }
             return result_dict(r);
           })
      .def("download",
           [](GpuGroup& g, int rank, int which) {
             auto v = g.rank(rank).download(which);
             return darr(static_cast<py::ssize_t>(v.size()), v.data());
           },
           py::arg("rank"), py::arg("which") = 0)
      .def("field_hash", [](GpuGroup& g, int rank, int which) { return g.rank(rank).field_hash(which); },
           py::arg("rank"), py::arg("which") = 0)
      .def("layout", [](GpuGroup& g, int rank) { return g.rank(rank).layout(); })
      .def("dims", [](GpuGroup& g) { return g.rank(0).dims(); })
      .def("mode", [](GpuGroup& g) { return g.rank(0).mode(); })
      .def("temporal", [](GpuGroup& g) { return g.rank(0).options().temporal; },
           "pass depth every rank runs (the constructor lowers the requested depth where a schedule needs it)")
      .def("overlapped", [](GpuGroup& g) { return g.rank(0).overlapped(); })
      .def("comm_counts", &GpuGroup::comm_counts)
      .def("traffic",
           [](GpuGroup& g, int rank) {
             const GpuSolver::Traffic t = g.rank(rank).traffic();
             py::dict d;
             d["field_bytes"] = t.field_bytes;
             d["halo_bytes"] = t.halo_bytes;
             return d;
           },
           py::arg("rank"), "GpuSolver.traffic() of one rank (bytes per solve of the last run()'s schedule)")
      .def("set_state", [](GpuGroup& g, const darr& prev, const darr& cur, int n0) {
        const i64 n = g.rank(0).problem().N + 1;
        g.set_state(ro_ptr(prev, n * n * n, "prev"), ro_ptr(cur, n * n * n, "cur"), n0);
      }, py::arg("prev"), py::arg("cur"), py::arg("step"))
      .def_property_readonly("transport", &GpuGroup::transport)
      .def_property_readonly("graph_enabled", &GpuGroup::graph_enabled)
      .def_property_readonly("world", &GpuGroup::world);
}
