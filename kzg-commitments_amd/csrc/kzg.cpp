// C++ facade: the reference's kzg:: API (/root/reference/src/kzg.h) over the
// C ABI of libkzgx.so.  Host code here only validates arguments, converts
// byte formats and marshals; every field / group computation is a GPU call.
#include "../../include/kzg.h"

#include <algorithm>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <mutex>
#include <random>

#include "curve_consts.h"

namespace kzg {

int CURVE_ORDER_BYTES;

namespace {

int g_curve = KZGX_CURVE_BN254;
int g_device = 0;  // kzg::set_device
std::mutex g_mu;
// default contexts for the setup-independent poly ops, one per (curve,
// device), created on first use and kept until process exit: init() and
// set_device() only switch which one default_ctx() hands out, so a pointer
// another thread obtained earlier stays valid
std::map<std::pair<int, int>, kzgx_ctx*> g_ctxs;

void check(int rc, const char* where) {
  if (rc == KZGX_OK) return;
  std::string msg = std::string(where) + ": " + kzgx_strerror(rc);
  if (rc == KZGX_ERR_ARG || rc == KZGX_ERR_DEGREE) throw std::invalid_argument(msg);
  if (rc == KZGX_ERR_DIV_ZERO) throw std::domain_error(msg);
  throw std::runtime_error(msg);
}

kzgx_ctx* default_ctx() {
  std::lock_guard<std::mutex> lk(g_mu);
  kzgx_ctx*& c = g_ctxs[{g_curve, g_device}];
  if (!c) check(kzgx_create(&c, g_curve, g_device), "kzgx_create");
  return c;
}

// r as 64-bit limbs for the selected curve
std::array<uint64_t, 4> order() {
  const uint32_t* w = g_curve == KZGX_CURVE_BN254 ? kzgx::BN254Fr::P : kzgx::BLS12381Fr::P;
  std::array<uint64_t, 4> r{};
  for (int i = 0; i < 4; i++) r[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  return r;
}

bool geq(const std::array<uint64_t, 4>& a, const std::array<uint64_t, 4>& b) {
  for (int i = 3; i >= 0; i--)
    if (a[i] != b[i]) return a[i] > b[i];
  return true;
}

void sub_in(std::array<uint64_t, 4>& a, const std::array<uint64_t, 4>& b) {
  unsigned __int128 br = 0;
  for (int i = 0; i < 4; i++) {
    unsigned __int128 t = (unsigned __int128)a[i] - b[i] - br;
    a[i] = (uint64_t)t;
    br = (t >> 64) & 1;
  }
}

// x mod r for a 256-bit x (x < 2^256 < 8 r on both curves)
void reduce(std::array<uint64_t, 4>& a) {
  const auto r = order();
  while (geq(a, r)) sub_in(a, r);
}

int base_limbs() { return kzgx_base_limbs(g_curve); }
size_t mod_bytes() { return g_curve == KZGX_CURVE_BN254 ? 32 : 48; }

std::vector<uint64_t> flat(const std::vector<Fr>& P) {
  std::vector<uint64_t> out(4 * P.size());
  for (size_t i = 0; i < P.size(); i++) std::memcpy(&out[4 * i], P[i].v.data(), 32);
  return out;
}

G1 to_g1(const uint64_t* xy, int inf) {
  G1 g;
  const int nl = base_limbs();
  g.inf = inf != 0;
  if (!g.inf)
    for (int i = 0; i < nl; i++) {
      g.x[i] = xy[i];
      g.y[i] = xy[nl + i];
    }
  return g;
}

// ECP_toOctet(..., false): 0x04 || X || Y big-endian (util.cpp:78-96).
// Infinity: miracl's ECP_inf is (0, 1), so the octet is 04 || 0 || 1.
std::vector<uint8_t> ecp_serialize(const G1& g) {
  const size_t mb = mod_bytes();
  const int nl = base_limbs();
  std::vector<uint8_t> oct(1 + 2 * mb, 0);
  oct[0] = 0x04;
  std::array<uint64_t, 6> x = g.x, y = g.y;
  if (g.inf) {
    x.fill(0);
    y.fill(0);
    y[0] = 1;
  }
  for (size_t k = 0; k < mb; k++) {
    oct[1 + mb - 1 - k] = (uint8_t)(x[k / 8] >> (8 * (k % 8)));
    oct[1 + 2 * mb - 1 - k] = (uint8_t)(y[k / 8] >> (8 * (k % 8)));
  }
  (void)nl;
  std::vector<uint8_t> out(4);
  uint32_t len = (uint32_t)oct.size();
  std::memcpy(out.data(), &len, 4);
  out.insert(out.end(), oct.begin(), oct.end());
  return out;
}

// ECP2_toOctet(..., false): 0x04 || x || y, each Fp2 as imag || real,
// MODBYTES big-endian each (miracl-core's current FP2_toBytes order; recalled,
// version-dependent).  Infinity: ECP2_inf = (0, 1).
void put_be(uint8_t* dst, const uint64_t* limbs, size_t mb) {
  for (size_t k = 0; k < mb; k++) dst[mb - 1 - k] = (uint8_t)(limbs[k / 8] >> (8 * (k % 8)));
}
void get_be(const uint8_t* src, uint64_t* limbs, size_t mb) {
  for (size_t k = 0; k < mb; k++) limbs[k / 8] |= (uint64_t)src[mb - 1 - k] << (8 * (k % 8));
}

std::vector<uint8_t> ecp2_octet(const G2& g) {
  const size_t mb = mod_bytes();
  std::vector<uint8_t> oct(1 + 4 * mb, 0);
  oct[0] = 0x04;
  std::array<uint64_t, 6> x0 = g.x0, x1 = g.x1, y0 = g.y0, y1 = g.y1;
  if (g.inf) {
    x0.fill(0);
    x1.fill(0);
    y0.fill(0);
    y1.fill(0);
    y0[0] = 1;
  }
  put_be(&oct[1], x1.data(), mb);
  put_be(&oct[1 + mb], x0.data(), mb);
  put_be(&oct[1 + 2 * mb], y1.data(), mb);
  put_be(&oct[1 + 3 * mb], y0.data(), mb);
  return oct;
}

// G2 canonical words (x.re, x.im, y.re, y.im; base_limbs() each) <-> G2
G2 to_g2(const uint64_t* w, bool inf) {
  G2 g;
  const int nl = base_limbs();
  g.inf = inf;
  if (!inf)
    for (int i = 0; i < nl; i++) {
      g.x0[i] = w[i];
      g.x1[i] = w[nl + i];
      g.y0[i] = w[2 * nl + i];
      g.y1[i] = w[3 * nl + i];
    }
  return g;
}

// deserialize_ECP (util.cpp:98-115): anything that is not a valid on-curve
// octet decodes to infinity.  The on-curve test runs on the GPU (g1_sum of
// the single point is the identity iff the point is valid).
G1 ecp_deserialize(const std::vector<uint8_t>& bytes) {
  G1 inf;
  if (bytes.size() < 4) return inf;
  uint32_t len;
  std::memcpy(&len, bytes.data(), 4);
  const size_t mb = mod_bytes();
  if (len != 1 + 2 * mb || bytes.size() < 4 + len || bytes[4] != 0x04) return inf;
  G1 g;
  g.inf = false;
  for (size_t k = 0; k < mb; k++) {
    g.x[k / 8] |= (uint64_t)bytes[4 + 1 + mb - 1 - k] << (8 * (k % 8));
    g.y[k / 8] |= (uint64_t)bytes[4 + 1 + 2 * mb - 1 - k] << (8 * (k % 8));
  }
  // validity: the GPU sums [P] alone and returns it canonically only if P is
  // a proper curve point (coordinates < p and y^2 = x^3 + b)
  const int nl = base_limbs();
  std::vector<uint64_t> xy(2 * nl);
  for (int i = 0; i < nl; i++) {
    xy[i] = g.x[i];
    xy[nl + i] = g.y[i];
  }
  int ok = 0;
  check(kzgx_g1_validate(default_ctx(), xy.data(), &ok), "kzgx_g1_validate");
  return ok ? g : inf;
}

}  // namespace

// ---- Fr ---------------------------------------------------------------------
Fr::Fr(long x) {
  unsigned long m = x < 0 ? (unsigned long)(-(x + 1)) + 1ul : (unsigned long)x;
  v = {m, 0, 0, 0};
  reduce(v);
  if (x < 0 && !is_zero()) {
    auto r = order();
    sub_in(r, v);
    v = r;
  }
}

Fr Fr::from_le_bytes(const uint8_t* bytes, size_t n) {
  Fr f;
  // NTL ZZFromBytes then conv<ZZ_p>: reduce mod r; inputs here are <= 32 bytes
  std::array<uint64_t, 4> a{};
  for (size_t k = 0; k < n && k < 32; k++) a[k / 8] |= (uint64_t)bytes[k] << (8 * (k % 8));
  for (size_t k = 32; k < n; k++)
    if (bytes[k]) throw std::invalid_argument("Fr::from_le_bytes: value wider than 256 bits");
  reduce(a);
  f.v = a;
  return f;
}

std::vector<uint8_t> Fr::to_le_bytes() const {
  std::vector<uint8_t> out;
  for (int k = 0; k < 32; k++) out.push_back((uint8_t)(v[k / 8] >> (8 * (k % 8))));
  while (!out.empty() && out.back() == 0) out.pop_back();  // NumBytes
  return out;
}

// ---- init -------------------------------------------------------------------
void init() { init(KZGX_CURVE_BN254); }

void init(int curve) {
  if (curve != KZGX_CURVE_BN254 && curve != KZGX_CURVE_BLS12381) throw std::invalid_argument("unknown curve");
  int dev;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_curve = curve;
    CURVE_ORDER_BYTES = 32;  // NumBytes(r) on both curves (trusted_setup.cpp:18)
    dev = g_device;
  }
  // the reference's init sets up its curve state before any other call
  // (src/kzg.h:33-38); here that is the device: HIP, every code object and
  // the generator tables, so no later call pays them.  Without a gfx950
  // device init still succeeds and the first GPU call throws.
  const int rc = kzgx_init_device(curve, dev);
  if (rc == KZGX_ERR_NO_DEVICE) return;
  check(rc, "kzgx_init_device");
  (void)default_ctx();
}

int curve() { return g_curve; }

void set_device(int device) {
  if (device < 0) throw std::invalid_argument("negative device ordinal");
  std::lock_guard<std::mutex> lk(g_mu);
  g_device = device;
}

int device() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_device;
}

// ---- blob -------------------------------------------------------------------
blob blob::from_string(std::string s) { return from_string(s, 0); }

blob blob::from_string(std::string s, int offset) {
  std::vector<std::pair<Fr, Fr>> d;
  d.reserve(s.size());
  for (size_t i = 0; i < s.size(); i++) d.push_back({Fr((long)i + offset), Fr((long)(signed char)s[i])});
  return blob(d);
}

blob blob::from_bytes(const uint8_t* bytes, int byte_offset, int byte_length, int chunk_size) {
  if (chunk_size > MAX_CHUNK_BYTES) throw std::invalid_argument("chunk_size must be at most MAX_CHUNK_BYTES.");
  if (chunk_size < 1) throw std::invalid_argument("chunk_size must be at least 1.");  // reference: UB
  if (byte_offset % chunk_size != 0) throw std::invalid_argument("byte_offset is not a multiple of chunk_size.");
  if (byte_length % chunk_size != 0) throw std::invalid_argument("byte_length is not a multiple of chunk_size.");
  const int chunk_offset = byte_offset / chunk_size;
  const int chunk_length = byte_length / chunk_size;
  std::vector<std::pair<Fr, Fr>> d;
  for (int i = 0; i < chunk_length; i++)
    d.push_back({Fr((long)chunk_offset + i), Fr::from_le_bytes(bytes + (size_t)i * chunk_size, chunk_size)});
  return blob(d);
}

// ---- poly -------------------------------------------------------------------
poly::poly(std::vector<Fr> _data) : data(std::move(_data)) {
  while (!data.empty() && data.back().is_zero()) data.pop_back();
}

poly poly::from_blob(blob b) {
  auto& pts = b.get_data();
  if (pts.empty()) return poly({});
  std::vector<uint64_t> xs(4 * pts.size()), ys(4 * pts.size()), c(4 * pts.size());
  for (size_t i = 0; i < pts.size(); i++) {
    std::memcpy(&xs[4 * i], pts[i].first.v.data(), 32);
    std::memcpy(&ys[4 * i], pts[i].second.v.data(), 32);
  }
  check(kzgx_poly_interpolate(default_ctx(), xs.data(), ys.data(), pts.size(), c.data()), "kzgx_poly_interpolate");
  std::vector<Fr> P(pts.size());
  for (size_t i = 0; i < pts.size(); i++) std::memcpy(P[i].v.data(), &c[4 * i], 32);
  return poly(P);
}

// serialize_ZZ_pX (util.cpp:118-140): i64 degree, then per coefficient a u8
// byte count and the minimal little-endian bytes
std::vector<uint8_t> poly::serialize() {
  std::vector<uint8_t> out(8);
  int64_t d = degree();
  std::memcpy(out.data(), &d, 8);
  for (auto& c : data) {
    auto b = c.to_le_bytes();
    out.push_back((uint8_t)b.size());
    out.insert(out.end(), b.begin(), b.end());
  }
  return out;
}

poly poly::deserialize(const std::vector<uint8_t>& bytes) {
  if (bytes.size() < 8) throw std::invalid_argument("poly::deserialize: truncated");
  int64_t d;
  std::memcpy(&d, bytes.data(), 8);
  size_t off = 8;
  std::vector<Fr> P;
  for (int64_t i = 0; i <= d; i++) {
    if (off >= bytes.size()) throw std::invalid_argument("poly::deserialize: truncated");
    uint8_t nb = bytes[off++];
    if (off + nb > bytes.size()) throw std::invalid_argument("poly::deserialize: truncated");
    P.push_back(Fr::from_le_bytes(bytes.data() + off, nb));
    off += nb;
  }
  return poly(P);
}

// ---- commit / proof ---------------------------------------------------------
std::vector<uint8_t> commit::serialize() { return ecp_serialize(curve_point); }
commit commit::deserialize(const std::vector<uint8_t>& b) { return commit(ecp_deserialize(b)); }
std::vector<uint8_t> proof::serialize() { return ecp_serialize(curve_point); }
proof proof::deserialize(const std::vector<uint8_t>& b) { return proof(ecp_deserialize(b)); }

// ---- trusted_setup ----------------------------------------------------------
trusted_setup::trusted_setup(int num_coeff) {
  if (num_coeff < 2) throw std::invalid_argument("num_coeff must be at least 2");
  // generate_random_BIG (util.cpp:62-76): 32 bytes from std::random_device, mod r
  std::random_device rd;
  uint8_t seed[32];
  for (auto& b : seed) b = (uint8_t)rd();
  Fr tau = Fr::from_le_bytes(seed, 32);
  check(kzgx_create(&ctx, g_curve, device()), "kzgx_create");
  check(kzgx_gen_srs_g1(ctx, tau.v.data(), 0, (size_t)num_coeff), "kzgx_gen_srs_g1");
  check(kzgx_gen_srs_g2(ctx, tau.v.data(), 0, (size_t)num_coeff), "kzgx_gen_srs_g2");
  n = (size_t)num_coeff;
  tau.v.fill(0);
  std::memset(seed, 0, sizeof seed);  // tau is toxic waste; the reference discards it too
}

trusted_setup::trusted_setup(int num_coeff, const Fr& tau) {
  if (num_coeff < 2) throw std::invalid_argument("num_coeff must be at least 2");
  check(kzgx_create(&ctx, g_curve, device()), "kzgx_create");
  check(kzgx_gen_srs_g1(ctx, tau.v.data(), 0, (size_t)num_coeff), "kzgx_gen_srs_g1");
  check(kzgx_gen_srs_g2(ctx, tau.v.data(), 0, (size_t)num_coeff), "kzgx_gen_srs_g2");
  n = (size_t)num_coeff;
}

trusted_setup::trusted_setup(const std::string& filename) {
  std::ifstream f(filename, std::ios::in | std::ios::binary);
  if (!f.is_open()) throw std::runtime_error("could not open trusted setup file");
  uint64_t num = 0;
  f.read(reinterpret_cast<char*>(&num), 8);
  if (!f || num == 0 || num > (1ull << 31)) throw std::runtime_error("bad trusted setup file");
  const size_t mb = mod_bytes();
  const int nl = base_limbs();
  std::vector<uint64_t> xy(2 * nl * num, 0);
  std::vector<uint8_t> one;
  for (uint64_t i = 0; i < num; i++) {
    uint32_t len = 0;
    f.read(reinterpret_cast<char*>(&len), 4);
    // the reference reads len bytes into a fixed buffer without a check
    // (trusted_setup.cpp:93-94); we reject anything but the uncompressed octet
    if (!f || len != 1 + 2 * mb) throw std::runtime_error("bad trusted setup file");
    std::vector<uint8_t> rec(4 + len);
    std::memcpy(rec.data(), &len, 4);
    f.read(reinterpret_cast<char*>(rec.data() + 4), len);
    if (!f) throw std::runtime_error("bad trusted setup file");
    G1 g = ecp_deserialize(rec);
    if (g.inf) throw std::runtime_error("bad trusted setup file");
    for (int k = 0; k < nl; k++) {
      xy[2 * nl * i + k] = g.x[k];
      xy[2 * nl * i + nl + k] = g.y[k];
    }
  }
  // G2 records (trusted_setup.cpp:103-118); a bad one is a logic_error there
  std::vector<uint64_t> xy2(4 * nl * num, 0);
  for (uint64_t i = 0; i < num; i++) {
    uint32_t len = 0;
    f.read(reinterpret_cast<char*>(&len), 4);
    if (!f || len != 1 + 4 * mb) throw std::logic_error("bad trusted setup file");
    std::vector<uint8_t> oct(len);
    f.read(reinterpret_cast<char*>(oct.data()), len);
    if (!f || oct[0] != 0x04) throw std::logic_error("bad trusted setup file");
    uint64_t* w = &xy2[4 * nl * i];
    get_be(&oct[1], w + nl, mb);           // x.im
    get_be(&oct[1 + mb], w, mb);           // x.re
    get_be(&oct[1 + 2 * mb], w + 3 * nl, mb);  // y.im
    get_be(&oct[1 + 3 * mb], w + 2 * nl, mb);  // y.re
  }
  check(kzgx_create(&ctx, g_curve, device()), "kzgx_create");
  std::vector<int> ok(num, 0);
  check(kzgx_g2_validate(ctx, xy2.data(), num, ok.data()), "kzgx_g2_validate");
  for (uint64_t i = 0; i < num; i++)
    if (!ok[i]) {
      kzgx_destroy(ctx);
      ctx = nullptr;
      throw std::logic_error("bad trusted setup file");
    }
  check(kzgx_load_srs_g1(ctx, xy.data(), num), "kzgx_load_srs_g1");
  check(kzgx_load_srs_g2(ctx, xy2.data(), num), "kzgx_load_srs_g2");
  n = num;
}

trusted_setup::~trusted_setup() {
  if (ctx) kzgx_destroy(ctx);
}

trusted_setup::trusted_setup(trusted_setup&& o) noexcept : ctx(o.ctx), n(o.n) {
  o.ctx = nullptr;
  o.n = 0;
}

trusted_setup& trusted_setup::operator=(trusted_setup&& o) noexcept {
  if (this != &o) {
    if (ctx) kzgx_destroy(ctx);
    ctx = o.ctx;
    n = o.n;
    o.ctx = nullptr;
    o.n = 0;
  }
  return *this;
}

G1 trusted_setup::polyeval_G1(const std::vector<Fr>& P) {
  if (P.empty()) return G1();  // deg -1 -> ECP_inf (trusted_setup.cpp:150-154)
  auto s = flat(P);
  std::vector<uint64_t> out(2 * base_limbs());
  int inf = 1;
  check(kzgx_msm_g1(ctx, s.data(), P.size(), out.data(), &inf), "kzgx_msm_g1");
  return to_g1(out.data(), inf);
}

commit trusted_setup::create_commit(const kzg::poly& p) {
  if (p.degree() + 1 >= (long)n)
    throw std::invalid_argument("polynomial degree be at most one less than the setup size (num_coeffs)");
  return commit(polyeval_G1(p.get_poly()));
}

bool trusted_setup::verify_commit(kzg::commit& c, const kzg::poly& p) {
  commit expected = create_commit(p);
  return c.get_curve_point() == expected.get_curve_point();
}

proof trusted_setup::create_proof(const kzg::poly& p, int byte_offset, int byte_length, int chunk_size) {
  if (chunk_size > MAX_CHUNK_BYTES) throw std::invalid_argument("chunk_size must at most MAX_CHUNK_BYTES.");
  if (chunk_size < 1) throw std::invalid_argument("chunk_size must be at least 1.");
  if (byte_offset % chunk_size != 0) throw std::invalid_argument("byte_offset is not a multiple of chunk_size.");
  if (byte_length % chunk_size != 0) throw std::invalid_argument("byte_length is not a multiple of chun_size.");
  return create_proof(p, byte_offset / chunk_size, byte_length / chunk_size);
}

proof trusted_setup::create_proof(const kzg::poly& p, int chunk_offset, int chunk_length) {
  if (chunk_length < 1) throw std::invalid_argument("chunk_length must be 1 or greater");
  const auto& P = p.get_poly();
  // the reference reads past _G1 here (UB) when deg q >= size; we refuse
  if ((long)P.size() - chunk_length > (long)n)
    throw std::invalid_argument("polynomial degree be at most one less than the setup size (num_coeffs)");
  auto c = flat(P);
  std::vector<uint64_t> out(2 * base_limbs());
  int inf = 1;
  if (chunk_length == 1) {
    Fr z((long)chunk_offset);
    uint64_t y[4];
    if (P.empty()) return proof(G1());
    check(kzgx_prove_single_batch(ctx, c.data(), P.size(), 0, z.v.data(), 1, out.data(), &inf, y),
          "kzgx_prove_single_batch");
    return proof(to_g1(out.data(), inf));
  }
  std::vector<uint64_t> xs(4 * (size_t)chunk_length);
  for (int i = 0; i < chunk_length; i++) {
    Fr x((long)chunk_offset + i);
    std::memcpy(&xs[4 * (size_t)i], x.v.data(), 32);
  }
  check(kzgx_prove_range(ctx, P.empty() ? nullptr : c.data(), P.size(), xs.data(), (size_t)chunk_length, out.data(),
                         &inf),
        "kzgx_prove_range");
  return proof(to_g1(out.data(), inf));
}

bool trusted_setup::verify_proof(commit& c, proof& pf, blob& expected_data) {
  auto& pts = expected_data.get_data();
  if (pts.size() < 1) throw std::invalid_argument("expected_data size must be 1 or greater");
  if (pts.size() >= n) return false;
  const int nl = base_limbs();
  std::vector<uint64_t> cxy(2 * nl, 0), pxy(2 * nl, 0), xs(4 * pts.size()), ys(4 * pts.size());
  const G1& cg = c.get_curve_point();
  const G1& pg = pf.get_curve_point();
  for (int i = 0; i < nl; i++) {
    cxy[i] = cg.x[i];
    cxy[nl + i] = cg.y[i];
    pxy[i] = pg.x[i];
    pxy[nl + i] = pg.y[i];
  }
  for (size_t j = 0; j < pts.size(); j++) {
    std::memcpy(&xs[4 * j], pts[j].first.v.data(), 32);
    std::memcpy(&ys[4 * j], pts[j].second.v.data(), 32);
  }
  int ok = 0;
  check(kzgx_verify_proof(ctx, cxy.data(), cg.inf ? 1 : 0, pxy.data(), pg.inf ? 1 : 0, xs.data(), ys.data(),
                          pts.size(), &ok),
        "kzgx_verify_proof");
  return ok != 0;
}

void trusted_setup::export_setup(const std::string& filename) {
  std::ofstream file(filename, std::ios::out | std::ios::binary | std::ios::trunc);
  if (!file.is_open()) {
    std::cerr << "failed to export" << std::endl;
    return;
  }
  const uint64_t num = n;
  file.write(reinterpret_cast<const char*>(&num), 8);
  for (const G1& g : g1_points()) {
    auto rec = ecp_serialize(g);  // u32 len || octet
    file.write(reinterpret_cast<const char*>(rec.data()), (std::streamsize)rec.size());
  }
  for (const G2& g : g2_points()) {
    auto oct = ecp2_octet(g);
    const uint32_t len = (uint32_t)oct.size();
    file.write(reinterpret_cast<const char*>(&len), 4);
    file.write(reinterpret_cast<const char*>(oct.data()), (std::streamsize)oct.size());
  }
}

std::vector<commit> trusted_setup::create_commits(const std::vector<kzg::poly>& polys) {
  std::vector<commit> res;
  if (polys.empty()) return res;
  size_t m = 0;
  for (auto& p : polys) {
    if (p.degree() + 1 >= (long)n)
      throw std::invalid_argument("polynomial degree be at most one less than the setup size (num_coeffs)");
    m = std::max(m, p.get_poly().size());
  }
  if (m == 0) return std::vector<commit>(polys.size(), commit(G1()));
  std::vector<uint64_t> s(4 * m * polys.size(), 0);  // zero-padded to a common length
  for (size_t b = 0; b < polys.size(); b++) {
    auto f = flat(polys[b].get_poly());
    std::memcpy(&s[4 * m * b], f.data(), f.size() * 8);
  }
  const int nl = base_limbs();
  std::vector<uint64_t> out(2 * nl * polys.size());
  std::vector<int> inf(polys.size());
  check(kzgx_msm_g1_batch(ctx, s.data(), m, polys.size(), out.data(), inf.data()), "kzgx_msm_g1_batch");
  for (size_t b = 0; b < polys.size(); b++) res.push_back(commit(to_g1(&out[2 * nl * b], inf[b])));
  return res;
}

std::vector<proof> trusted_setup::create_proofs(const kzg::poly& p, const std::vector<long>& points) {
  std::vector<proof> res;
  const auto& P = p.get_poly();
  if (points.empty()) return res;
  if (P.empty()) return std::vector<proof>(points.size(), proof(G1()));
  if ((long)P.size() - 1 > (long)n)
    throw std::invalid_argument("polynomial degree be at most one less than the setup size (num_coeffs)");
  auto c = flat(P);
  std::vector<uint64_t> zs(4 * points.size());
  for (size_t j = 0; j < points.size(); j++) {
    Fr z(points[j]);
    std::memcpy(&zs[4 * j], z.v.data(), 32);
  }
  const int nl = base_limbs();
  std::vector<uint64_t> out(2 * nl * points.size());
  std::vector<int> inf(points.size());
  check(kzgx_prove_single_batch(ctx, c.data(), P.size(), 0, zs.data(), points.size(), out.data(), inf.data(),
                                nullptr),
        "kzgx_prove_single_batch");
  for (size_t j = 0; j < points.size(); j++) res.push_back(proof(to_g1(&out[2 * nl * j], inf[j])));
  return res;
}

std::vector<bool> trusted_setup::verify_proofs(std::vector<commit>& commits, std::vector<proof>& proofs,
                                              const std::vector<std::pair<Fr, Fr>>& points) {
  const size_t m = commits.size();
  if (proofs.size() != m || points.size() != m) throw std::invalid_argument("verify_proofs: size mismatch");
  std::vector<bool> res(m, false);
  if (m == 0) return res;
  const int nl = base_limbs();
  std::vector<uint64_t> c(2 * nl * m, 0), p(2 * nl * m, 0), z(4 * m), y(4 * m);
  std::vector<int> ci(m), pi(m), ok(m);
  for (size_t k = 0; k < m; k++) {
    const G1& cg = commits[k].get_curve_point();
    const G1& pg = proofs[k].get_curve_point();
    for (int i = 0; i < nl; i++) {
      c[2 * nl * k + i] = cg.x[i];
      c[2 * nl * k + nl + i] = cg.y[i];
      p[2 * nl * k + i] = pg.x[i];
      p[2 * nl * k + nl + i] = pg.y[i];
    }
    ci[k] = cg.inf;
    pi[k] = pg.inf;
    std::memcpy(&z[4 * k], points[k].first.v.data(), 32);
    std::memcpy(&y[4 * k], points[k].second.v.data(), 32);
  }
  check(kzgx_verify_single_batch(ctx, c.data(), ci.data(), p.data(), pi.data(), z.data(), y.data(), m, ok.data()),
        "kzgx_verify_single_batch");
  for (size_t k = 0; k < m; k++) res[k] = ok[k] != 0;
  return res;
}

std::vector<G1> trusted_setup::g1_points() const {
  const int nl = base_limbs();
  std::vector<uint64_t> xy(2 * nl * n);
  check(kzgx_get_srs_g1(ctx, xy.data(), n), "kzgx_get_srs_g1");
  std::vector<G1> res;
  for (size_t i = 0; i < n; i++) {
    bool z = true;
    for (int k = 0; k < 2 * nl; k++) z &= xy[2 * nl * i + k] == 0;
    res.push_back(to_g1(&xy[2 * nl * i], z));
  }
  return res;
}

void trusted_setup::precompute(int window_bits, size_t points) {
  check(kzgx_set_fixed_base(ctx, window_bits, window_bits ? (points ? std::min(points, n) : n) : 0),
        "kzgx_set_fixed_base");
}

void trusted_setup::default_table(int window_bits, size_t points) {
  check(kzgx_set_default_table(ctx, window_bits, window_bits ? points : 0), "kzgx_set_default_table");
}

int trusted_setup::precompute_budget(size_t budget_bytes, size_t points) {
  int c = 0;
  check(kzgx_set_fixed_base_budget(ctx, budget_bytes, points ? std::min(points, n) : n, &c),
        "kzgx_set_fixed_base_budget");
  return c;
}

std::vector<G2> trusted_setup::g2_points() const {
  const int nl = base_limbs();
  const size_t n2 = kzgx_srs_g2_size(ctx);
  std::vector<uint64_t> xy(4 * nl * n2);
  if (n2) check(kzgx_get_srs_g2(ctx, xy.data(), n2), "kzgx_get_srs_g2");
  std::vector<G2> res;
  for (size_t i = 0; i < n2; i++) {
    bool z = true;
    for (int k = 0; k < 4 * nl; k++) z &= xy[4 * nl * i + k] == 0;
    res.push_back(to_g2(&xy[4 * nl * i], z));
  }
  return res;
}

}  // namespace kzg
