// The reference's benchmark (benchmark/benchmark.cpp) on the C++ facade:
// the same timed regions -- kzg::trusted_setup(max_degree) for 128..4096
// terms, then on a 5000-point setup one create_commit / create_proof(poly,
// 0, 1) / verify_proof per degree 128..4096, and create_proof(poly, 0, N) /
// verify_proof for N = 128..4096 -- each a single call with host buffers,
// timed with std::chrono around the call exactly as the reference does.
// Polynomials come from random strings through blob::from_string and
// poly::from_blob, as in the reference.  Each region is also repeated
// (median of 9) after its first call, since a first call on a fresh setup
// includes one-time work (kernel code-object loads, workspace growth).
// Prints the reference's table and one JSON line.
//
//   kzg_bench [--json-only] [--curve BN254|BLS12381]
//
// The reference builds this benchmark once per curve (benchmark_curves.sh:
// 43-51 rebuilds it with each miracl curve config); here the curve is the
// run-time argument of kzg::init.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <iostream>
#include <random>
#include <string>
#include <vector>

#include "kzg.h"

using clk = std::chrono::steady_clock;

static std::string random_string(int length, std::mt19937& gen) {
  static const std::string chars = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz";
  std::uniform_int_distribution<> d(0, (int)chars.size() - 1);
  std::string s;
  s.reserve(length);
  for (int i = 0; i < length; i++) s += chars[d(gen)];
  return s;
}

template <class F>
static double ms_of(F&& f) {
  const auto t0 = clk::now();
  f();
  return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

template <class F>
static double median_ms(F&& f, int reps = 9) {
  std::vector<double> v;
  for (int i = 0; i < reps; i++) v.push_back(ms_of(f));
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  bool json_only = false;
  int curve = KZGX_CURVE_BN254;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    if (a == "--json-only") {
      json_only = true;
    } else if (a == "--curve" && i + 1 < argc) {
      const std::string c = argv[++i];
      if (c == "BN254") curve = KZGX_CURVE_BN254;
      else if (c == "BLS12381" || c == "BLS12-381") curve = KZGX_CURVE_BLS12381;
      else {
        std::fprintf(stderr, "kzg_bench: unknown curve %s (BN254 or BLS12381)\n", c.c_str());
        return 2;
      }
    } else {
      std::fprintf(stderr, "usage: kzg_bench [--json-only] [--curve BN254|BLS12381]\n");
      return 2;
    }
  }
  kzg::init(curve);
  if (!json_only) std::printf("curve: %s\n", curve == KZGX_CURVE_BN254 ? "BN254" : "BLS12381");
  std::mt19937 gen(0x4B5A47);
  std::string js = std::string("{\"curve\": \"") + (curve == KZGX_CURVE_BN254 ? "BN254" : "BLS12381") +
                   "\", \"setup_ms\": {";
  if (!json_only) std::cout << "=== Benchmarking Trusted Setup ===" << std::endl;
  for (int max_degree = 128; max_degree <= 4096; max_degree *= 2) {
    const double t = ms_of([&] { kzg::trusted_setup s(max_degree); });
    if (!json_only) std::printf("Terms: %4d | Setup: %8.3fms\n", max_degree, t);
    js += (max_degree > 128 ? ", \"" : "\"") + std::to_string(max_degree) + "\": " + std::to_string(t);
  }
  js += "}, \"single\": {";
  kzg::trusted_setup kzg(5000);
  if (!json_only) std::cout << "\n=== Benchmarking Single Proofs ===" << std::endl;
  bool all_ok = true;
  for (int degree = 128; degree <= 4096; degree *= 2) {
    const std::string data = random_string(degree + 1, gen);
    kzg::blob b = kzg::blob::from_string(data);
    kzg::poly p = kzg::poly::from_blob(b);
    kzg::commit c({});
    kzg::proof pr({});
    const double tc = ms_of([&] { c = kzg.create_commit(p); });
    const double tp = ms_of([&] { pr = kzg.create_proof(p, 0, 1); });
    kzg::blob target = kzg::blob::from_string(data.substr(0, 1), 0);
    bool ok = false;
    const double tv = ms_of([&] { ok = kzg.verify_proof(c, pr, target); });
    all_ok = all_ok && ok;
    const double mc = median_ms([&] { c = kzg.create_commit(p); });
    const double mp = median_ms([&] { pr = kzg.create_proof(p, 0, 1); });
    const double mv = median_ms([&] { ok = kzg.verify_proof(c, pr, target); });
    all_ok = all_ok && ok;
    if (!json_only)
      std::printf("Degree: %8d | Commit: %10.3fms | Proof: %10.3fms | Verify: %10.3fms | %s   (median: %.3f / %.3f / %.3f ms)\n",
                  degree, tc, tp, tv, ok ? "ok" : "FAIL", mc, mp, mv);
    char buf[256];
    std::snprintf(buf, sizeof buf,
                  "%s\"%d\": {\"commit_ms\": %.4f, \"proof_ms\": %.4f, \"verify_ms\": %.4f, \"median_commit_ms\": %.4f, "
                  "\"median_proof_ms\": %.4f, \"median_verify_ms\": %.4f, \"verified\": %s}",
                  degree > 128 ? ", " : "", degree, tc, tp, tv, mc, mp, mv, ok ? "true" : "false");
    js += buf;
  }
  js += "}, \"multi\": {";
  if (!json_only) std::cout << "\n=== Benchmarking Multi Proofs ===" << std::endl;
  const std::string data = random_string(4096, gen);
  kzg::blob b = kzg::blob::from_string(data);
  kzg::poly p = kzg::poly::from_blob(b);
  kzg::commit c = kzg.create_commit(p);
  for (int num = 128; num <= 4096; num *= 2) {
    kzg::proof pr({});
    const double tp = ms_of([&] { pr = kzg.create_proof(p, 0, num); });
    kzg::blob target = kzg::blob::from_string(data.substr(0, num), 0);
    bool ok = false;
    const double tv = ms_of([&] { ok = kzg.verify_proof(c, pr, target); });
    all_ok = all_ok && ok;
    const double mp = median_ms([&] { pr = kzg.create_proof(p, 0, num); }, 5);
    if (!json_only)
      std::printf("Degree: %3d | Proofs: %7d | Proof: %7.3fms | Verify: %7.3fms | %s   (median proof %.3f ms)\n", 4096,
                  num, tp, tv, ok ? "ok" : "FAIL", mp);
    char buf[200];
    std::snprintf(buf, sizeof buf, "%s\"%d\": {\"proof_ms\": %.4f, \"verify_ms\": %.4f, \"median_proof_ms\": %.4f, \"verified\": %s}",
                  num > 128 ? ", " : "", num, tp, tv, mp, ok ? "true" : "false");
    js += buf;
  }
  js += std::string("}, \"all_verified\": ") + (all_ok ? "true" : "false") + "}";
  std::cout << js << std::endl;
  return all_ok ? 0 : 1;
}
