// kzg_cli -- command-line driver over the kzg:: facade (include/kzg.h), the
// counterpart of the reference's demo/shared/kzg-cli.cpp:28-109.  Same four
// verbs, same stdout formats and exit codes, so the reference's demo scripts
// can call it unchanged; every commitment / proof / pairing runs on the GPU.
//
//   kzg_cli setup  <num_coeff>                    writes the setup file
//   kzg_cli commit <file>                         prints the commitment (hex)
//   kzg_cli prove  <file> <seed>                  prints "<proof hex> <chunk> <data hex>"
//   kzg_cli verify <commit hex> <proof hex> <chunk> <data hex>   exit 0 = valid, 1 = invalid
//
// Options (extensions): --setup <path> (default ../shared/kzg_public, as in
// the reference), --curve 0|1 (BN254 default, BLS12-381).
#include <kzg.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <iterator>
#include <string>
#include <vector>

namespace {

std::string g_setup = "../shared/kzg_public";

std::string hexstr(const std::vector<uint8_t>& b) {
  static const char* d = "0123456789abcdef";
  std::string s;
  s.reserve(2 * b.size());
  for (uint8_t x : b) {
    s.push_back(d[x >> 4]);
    s.push_back(d[x & 15]);
  }
  return s;
}

std::vector<uint8_t> unhex(const std::string& s) {
  std::vector<uint8_t> out;
  for (size_t i = 0; i < s.size(); i += 2) out.push_back((uint8_t)std::strtol(s.substr(i, 2).c_str(), nullptr, 16));
  return out;
}

std::vector<uint8_t> slurp(const std::string& path) {
  std::ifstream f(path, std::ios::in | std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + path);
  return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}

// pad to a whole number of chunks: always appends 1..chunk bytes of zeros,
// like kzg-cli.cpp:42-46
void pad_chunks(std::vector<uint8_t>& bytes) {
  const int cs = MAX_CHUNK_BYTES;
  const int pad = cs - (int)(bytes.size() % cs);
  bytes.insert(bytes.end(), (size_t)pad, 0);
}

kzg::poly file_poly(std::vector<uint8_t>& bytes) {
  pad_chunks(bytes);
  return kzg::poly::from_blob(kzg::blob::from_bytes(bytes.data(), 0, (int)bytes.size(), MAX_CHUNK_BYTES));
}

int cmd_setup(int num_coeff) {
  const auto t0 = std::chrono::steady_clock::now();
  kzg::trusted_setup kzg(num_coeff);
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::cout << "KZG trusted setup generated in " << s << "s" << std::endl;
  std::cout << "  num_coeff=" << num_coeff << std::endl;
  std::cout << "  max_commit_bytes=" << (long)num_coeff * MAX_CHUNK_BYTES << std::endl;
  kzg.export_setup(g_setup);
  return 0;
}

int cmd_commit(const std::string& path) {
  kzg::trusted_setup kzg(g_setup);
  std::vector<uint8_t> bytes = slurp(path);
  kzg::poly poly = file_poly(bytes);
  std::cout << hexstr(kzg.create_commit(poly).serialize()) << std::endl;
  return 0;
}

int cmd_prove(const std::string& path, int seed) {
  kzg::trusted_setup kzg(g_setup);
  std::vector<uint8_t> bytes = slurp(path);
  const int chunks = (int)bytes.size() / MAX_CHUNK_BYTES;  // of the unpadded file (kzg-cli.cpp:75)
  kzg::poly poly = file_poly(bytes);
  if (chunks - 4 <= 0) throw std::invalid_argument("file too short for a 4-chunk proof");
  const int chunk = seed % (chunks - 4);
  kzg::proof proof = kzg.create_proof(poly, chunk, 4);
  std::vector<uint8_t> sub(bytes.begin() + (long)chunk * MAX_CHUNK_BYTES,
                           bytes.begin() + (long)(chunk + 4) * MAX_CHUNK_BYTES);
  std::cout << hexstr(proof.serialize()) << " " << chunk << " " << hexstr(sub) << std::endl;
  return 0;
}

int cmd_verify(const std::string& c_hex, const std::string& p_hex, int chunk, const std::string& d_hex) {
  kzg::trusted_setup kzg(g_setup);
  kzg::commit c = kzg::commit::deserialize(unhex(c_hex));
  kzg::proof p = kzg::proof::deserialize(unhex(p_hex));
  std::vector<uint8_t> data = unhex(d_hex);
  kzg::blob b = kzg::blob::from_bytes(data.data(), chunk * MAX_CHUNK_BYTES, 4 * MAX_CHUNK_BYTES, MAX_CHUNK_BYTES);
  return kzg.verify_proof(c, p, b) ? 0 : 1;
}

int usage() {
  std::cerr << "usage: kzg_cli [--setup path] [--curve 0|1] setup <n> | commit <file> | prove <file> <seed> | "
               "verify <commit> <proof> <chunk> <data>"
            << std::endl;
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<std::string> a;
  int curve = KZGX_CURVE_BN254;
  for (int i = 1; i < argc; i++) {
    std::string s = argv[i];
    if (s == "--setup" && i + 1 < argc) {
      g_setup = argv[++i];
    } else if (s == "--curve" && i + 1 < argc) {
      curve = std::atoi(argv[++i]);
    } else {
      a.push_back(s);
    }
  }
  if (a.empty()) return usage();
  try {
    kzg::init(curve);
    if (a[0] == "setup" && a.size() == 2) return cmd_setup(std::stoi(a[1]));
    if (a[0] == "commit" && a.size() == 2) return cmd_commit(a[1]);
    if (a[0] == "prove" && a.size() == 3) return cmd_prove(a[1], std::stoi(a[2]));
    if (a[0] == "verify" && a.size() == 5) return cmd_verify(a[1], a[2], std::stoi(a[3]), a[4]);
  } catch (const std::exception& e) {
    std::cerr << "kzg_cli: " << e.what() << std::endl;
    return 3;
  }
  return usage();
}
