/* kzg.h -- C++ API of the MI355X KZG engine, mirroring the reference's
 * public surface (/root/reference/src/kzg.h:27-292, namespace kzg) so a user
 * of uncommitted6453/kzg-commitments can switch by re-linking:
 *
 *   kzg::init                       src/kzg.h:38        trusted_setup.cpp:15-19
 *   kzg::blob::from_string/bytes    src/kzg.h:40-87     blob.cpp:3-48
 *   kzg::poly::from_blob/(de)ser.   src/kzg.h:89-125    poly.cpp:4-15, util.cpp:118-170
 *   kzg::commit / kzg::proof        src/kzg.h:127-180   commit.cpp, proof.cpp, util.cpp:78-115
 *   kzg::trusted_setup              src/kzg.h:182-290   trusted_setup.cpp:21-287
 *
 * Differences, all at the type level (semantics and error behaviour follow
 * the reference): NTL ZZ_p / ZZ_pX are replaced by kzg::Fr / std::vector<Fr>
 * (canonical residues mod r), miracl ECP by kzg::G1 (canonical affine
 * coordinates), and the curve is chosen at run time (kzg::init(curve))
 * instead of by rebuilding with another kzg_config.h.  Every group and
 * scalar-field computation runs on the GPU through the C ABI in kzg_gpu.h.
 */
#ifndef KZG_H
#define KZG_H

#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "kzg_gpu.h"

namespace kzg {

extern int CURVE_ORDER_BYTES;

#define MAX_CHUNK_BYTES (kzg::CURVE_ORDER_BYTES - 1)

/** Element of Z_r (the reference's NTL ZZ_p under ZZ_p::init(r)). */
struct Fr {
  std::array<uint64_t, 4> v{};  // little-endian limbs, always < r
  Fr() = default;
  /** integer -> residue, like NTL `ZZ_p x; x = long` (negative -> r - |x|) */
  Fr(long x);
  /** little-endian bytes -> residue (NTL ZZFromBytes + conv<ZZ_p>) */
  static Fr from_le_bytes(const uint8_t* bytes, size_t n);
  /** minimal little-endian encoding (NTL BytesFromZZ with NumBytes) */
  std::vector<uint8_t> to_le_bytes() const;
  bool is_zero() const { return (v[0] | v[1] | v[2] | v[3]) == 0; }
  bool operator==(const Fr& o) const { return v == o.v; }
  bool operator!=(const Fr& o) const { return v != o.v; }
};

/** Affine G1 point (the reference's miracl ECP); canonical coordinates. */
struct G1 {
  std::array<uint64_t, 6> x{}, y{};  // 4 limbs used on BN254, 6 on BLS12-381
  bool inf = true;
  bool operator==(const G1& o) const { return inf == o.inf && (inf || (x == o.x && y == o.y)); }
  bool operator!=(const G1& o) const { return !(*this == o); }
};

/** Affine G2 point on the sextic twist (the reference's miracl ECP2):
 *  x = x0 + x1 i, y = y0 + y1 i, canonical coordinates. */
struct G2 {
  std::array<uint64_t, 6> x0{}, x1{}, y0{}, y1{};
  bool inf = true;
  bool operator==(const G2& o) const {
    return inf == o.inf && (inf || (x0 == o.x0 && x1 == o.x1 && y0 == o.y0 && y1 == o.y1));
  }
  bool operator!=(const G2& o) const { return !(*this == o); }
};

/** Initialize the library (BN254, the reference's default build). */
void init();
/** Extension: pick the curve at run time (KZGX_CURVE_BN254 / KZGX_CURVE_BLS12381). */
void init(int curve);
/** Curve selected by init(). */
int curve();
/** Extension: the GPU (HIP device ordinal) that trusted_setups constructed
 *  after this call, and the setup-independent polynomial helpers, run on
 *  (default 0).  One process per GPU is the multi-GPU model; a process may
 *  also hold setups on several devices.  @throws std::invalid_argument for a
 *  negative ordinal (a missing device fails at the next construction). */
void set_device(int device);
int device();

class blob {
 private:
  std::vector<std::pair<Fr, Fr>> data;

 public:
  blob(std::vector<std::pair<Fr, Fr>>& _data) : data(_data) {}
  std::vector<std::pair<Fr, Fr>>& get_data() { return data; }
  /** points (i + offset, (signed char) s[i]) (blob.cpp:7-18) */
  static blob from_string(std::string s);
  static blob from_string(std::string s, int offset);
  /** little-endian chunk_size-byte chunks; x = byte_offset / chunk_size + i (blob.cpp:20-48)
   *  @throws std::invalid_argument on chunk_size / alignment violations */
  static blob from_bytes(const uint8_t* bytes, int byte_offset, int byte_length, int chunk_size);
};

class poly {
 private:
  std::vector<Fr> data;  // normalized: no trailing zero coefficient

 public:
  poly(std::vector<Fr> _data);
  const std::vector<Fr>& get_poly() const { return data; }
  /** NTL deg(): -1 for the zero polynomial */
  long degree() const { return (long)data.size() - 1; }
  /** interpolate the blob's points (polyfit, util.cpp:172-184) on the GPU */
  static poly from_blob(blob blob);
  std::vector<uint8_t> serialize();
  static poly deserialize(const std::vector<uint8_t>&);
};

class commit {
 private:
  G1 curve_point;

 public:
  commit(G1 _curve_point) : curve_point(_curve_point) {}
  G1& get_curve_point() { return curve_point; }
  std::vector<uint8_t> serialize();
  static commit deserialize(const std::vector<uint8_t>&);
};

class proof {
 private:
  G1 curve_point;

 public:
  proof(G1 _curve_point) : curve_point(_curve_point) {}
  G1& get_curve_point() { return curve_point; }
  std::vector<uint8_t> serialize();
  static proof deserialize(const std::vector<uint8_t>& bytes);
};

class trusted_setup {
 private:
  kzgx_ctx* ctx = nullptr;  // device SRS + stream + workspaces
  size_t n = 0;

  G1 polyeval_G1(const std::vector<Fr>& P);

 public:
  /** random tau (std::random_device), [tau^i]G1 and [tau^i]G2 for
   *  i < num_coeff, on the GPU  @throws std::invalid_argument if num_coeff < 2 */
  trusted_setup(int num_coeff);
  /** Extension: deterministic setup from a given tau (tests, benchmarks). */
  trusted_setup(int num_coeff, const Fr& tau);
  /** load a setup written by export_setup (trusted_setup.cpp:76-121)
   *  @throws std::runtime_error for an inaccessible file or a bad G1 record,
   *          std::logic_error for a bad G2 record (as the reference does) */
  trusted_setup(const std::string& filename);
  ~trusted_setup();
  trusted_setup(const trusted_setup&) = delete;
  trusted_setup& operator=(const trusted_setup&) = delete;
  trusted_setup(trusted_setup&& o) noexcept;
  trusted_setup& operator=(trusted_setup&& o) noexcept;

  size_t size() const { return n; }

  /** C = [P(s)]1  @throws std::invalid_argument if deg(P) + 1 >= size() */
  commit create_commit(const kzg::poly& poly);
  bool verify_commit(kzg::commit& commit, const kzg::poly& poly);
  /** @throws std::invalid_argument on chunk_size / alignment violations */
  proof create_proof(const kzg::poly& poly, int byte_offset, int byte_length, int chunk_size);
  /** @throws std::invalid_argument if chunk_length < 1 */
  proof create_proof(const kzg::poly& poly, int chunk_offset, int chunk_length);
  /** e(proof, [Z(s)]2) == e(C - [I(s)]1, [1]2), all on the GPU
   *  (trusted_setup.cpp:230-254)
   *  @throws std::invalid_argument if expected_data is empty; false if it
   *          holds >= size() points */
  bool verify_proof(commit& commit, proof& proof, blob& expected_data);
  /** writes the reference file layout (trusted_setup.cpp:256-287):
   *  u64 n, n x (u32 len, G1 octet), n x (u32 len, G2 octet); prints
   *  "failed to export" and returns if the file cannot be opened */
  void export_setup(const std::string& filename = "kzg_public");

  /** Extensions: batched commits / single-point openings in one GPU pass. */
  std::vector<commit> create_commits(const std::vector<kzg::poly>& polys);
  std::vector<proof> create_proofs(const kzg::poly& poly, const std::vector<long>& points);
  /** Extension: many single-point verify_proof calls in one GPU pass;
   *  result k == verify_proof(commits[k], proofs[k], blob {points[k]}). */
  std::vector<bool> verify_proofs(std::vector<commit>& commits, std::vector<proof>& proofs,
                                  const std::vector<std::pair<Fr, Fr>>& points);
  /** copy of the G1 / G2 SRS points */
  std::vector<G1> g1_points() const;
  std::vector<G2> g2_points() const;
  /** Extension: precompute the fixed-base table of odd multiples for the
   *  first `points` SRS points (0 = all) with `window_bits`-bit windows
   *  (kzgx_set_fixed_base).  Entries are 64 B (BN254) / 112 B (BLS12-381);
   *  over 4097 points BN254 c = 17 (15 windows, the bench's table) takes
   *  257.8 GB of HBM, c = 16 137.5 GB, c = 12 11.8 GB, and BLS12-381 c = 16
   *  240.6 GB.  Commits and proofs over that prefix then run as plain table
   *  sums.  window_bits = 0 drops the table.  Without it, batches run on
   *  the default table below. */
  void precompute(int window_bits = 16, size_t points = 0);
  /** Extension: the default table (kzgx_set_default_table), built with
   *  every setup: odd multiples of the first 4097 SRS points at the widest
   *  window c <= 12 that fits 4.5% of the HBM (window_bits = -1, the default:
   *  BN254 c = 12, 11.8 GB; BLS12-381 c = 11, 9.7 GB).  Single create_commit /
   *  create_proof calls of degree <= 4096 take its one-launch path, batches
   *  its batched kernel.  The reference's create_commit allocates nothing
   *  beyond the SRS (src/trusted_setup.cpp:137-142): default_table(0)
   *  restores that, and every MSM then runs the table-less Pippenger. */
  void default_table(int window_bits, size_t points = 4097);
  /** Extension: the widest window whose table over `points` SRS points
   *  (0 = all) fits `budget_bytes` and the free HBM; returns the window
   *  built (0: none fits, Pippenger stays).  DESIGN.md section 3 holds the
   *  measured throughput at each table size. */
  int precompute_budget(size_t budget_bytes, size_t points = 0);
};

}  // namespace kzg

#endif
