// gx_codec_host.hpp — host side of the full-state JSON codec: gx_set_names
// (encoded strings, map-key orders and lookup tables, built once), and the launch sequences of
// gx_local_state_json / gx_decode_state_json / gx_merge_remote_state_json (gx_codec.hpp).
// Included by gx_engine.hip after the engine's host helpers.
#pragma once
#include <algorithm>
#include <string>

// grow-only device buffer
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
};
static int dbuf(DevBuf &b, size_t bytes, void **out) {
  if (bytes > b.cap) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    size_t c = 1 << 16;
    while (c < bytes) c <<= 1;
    if (hipMalloc(&b.p, c) != hipSuccess) {
      (void)hipGetLastError();
      return GX_ENOMEM;
    }
    b.cap = c;
  }
  *out = b.p;
  return GX_OK;
}
// bump allocator over one grow-only buffer (all pieces of one phase of a call)
struct Bump {
  size_t off = 0;
  template <class T>
  T *take(char *base, size_t n) {
    off = (off + 255) & ~(size_t)255;
    T *p = (T *)(base + off);
    off += sizeof(T) * n;
    return p;
  }
};

// Device -> pageable host copy through two pinned staging chunks: the DMA of chunk i+1 overlaps
// the host memcpy of chunk i (a plain pageable hipMemcpy runs at a few GB/s).
#define PIN_CHUNK (8u << 20)
struct Pinned {
  char *p[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
};
static int d2h_staged(gx_engine *e, Pinned &pn, char *dst, const char *src, size_t n) {
  for (int i = 0; i < 2; i++) {
    if (!pn.p[i]) {
      HIPCHK(hipHostMalloc((void **)&pn.p[i], PIN_CHUNK, hipHostMallocDefault));
      HIPCHK(hipEventCreateWithFlags(&pn.ev[i], hipEventDisableTiming));
    }
  }
  const size_t nch = (n + PIN_CHUNK - 1) / PIN_CHUNK;
  for (size_t c = 0; c < nch && c < 2; c++) {
    const size_t len = std::min<size_t>(PIN_CHUNK, n - c * PIN_CHUNK);
    HIPCHK(hipMemcpyAsync(pn.p[c & 1], src + c * PIN_CHUNK, len, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipEventRecord(pn.ev[c & 1], e->stream));
  }
  for (size_t c = 0; c < nch; c++) {
    const size_t len = std::min<size_t>(PIN_CHUNK, n - c * PIN_CHUNK);
    HIPCHK(hipEventSynchronize(pn.ev[c & 1]));
    memcpy(dst + c * PIN_CHUNK, pn.p[c & 1], len);
    if (c + 2 < nch) {
      const size_t l2 = std::min<size_t>(PIN_CHUNK, n - (c + 2) * PIN_CHUNK);
      HIPCHK(hipMemcpyAsync(pn.p[c & 1], src + (c + 2) * PIN_CHUNK, l2, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipEventRecord(pn.ev[c & 1], e->stream));
    }
  }
  return GX_OK;
}

struct CodecState {
  Pinned pin2;                   // staging for LocalState copies to the caller
  gxc::Names nm;                 // device pointers
  std::vector<void *> owned;     // device allocations of the names tables
  std::vector<uint32_t> ehost_len;
  uint32_t *seen = nullptr;      // [R] duplicate record keys
  DevBuf out;                    // encoder output
  DevBuf enc;                    // encoder server lengths / offsets + scan scratch
  DevBuf in, ph1, ph2, ph3;      // decoder input and phase buffers
};

static void codec_free(gx_engine *e) {
  CodecState *c = e->codec;
  if (!c) return;
  for (void *p : c->owned) (void)hipFree(p);
  if (c->seen) (void)hipFree(c->seen);
  for (DevBuf *b : {&c->out, &c->enc, &c->in, &c->ph1, &c->ph2, &c->ph3})
    if (b->p) (void)hipFree(b->p);
  for (int i = 0; i < 2; i++) {
    if (c->pin2.p[i]) (void)hipHostFree(c->pin2.p[i]);
    if (c->pin2.ev[i]) (void)hipEventDestroy(c->pin2.ev[i]);
  }
  delete c;
  e->codec = nullptr;
}

// encoding/json encodeState.string(s, escapeHTML = true) (Go 1.13)
static void go_json_string(std::string &o, const char *s0, size_t n) {
  static const char hex[] = "0123456789abcdef";
  const uint8_t *s = (const uint8_t *)s0;
  o.push_back('"');
  size_t i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c < 0x80) {
      if (c >= 0x20 && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&') {
        o.push_back((char)c);
      } else {
        o.push_back('\\');
        if (c == '"' || c == '\\') o.push_back((char)c);
        else if (c == '\n') o.push_back('n');
        else if (c == '\r') o.push_back('r');
        else if (c == '\t') o.push_back('t');
        else {
          o += "u00";
          o.push_back(hex[c >> 4]);
          o.push_back(hex[c & 15]);
        }
      }
      i++;
      continue;
    }
    uint32_t sz;
    uint32_t r = gxc::utf8_rune(s + i, (uint32_t)std::min<size_t>(n - i, 4), sz);
    if (r == 0xFFFD && sz == 1) o += "\\ufffd";
    else if (r == 0x2028) o += "\\u2028";
    else if (r == 0x2029) o += "\\u2029";
    else o.append((const char *)s + i, sz);
    i += sz;
  }
  o.push_back('"');
}
static uint64_t fnv1a(const char *s, size_t n) {
  uint64_t h = 0xCBF29CE484222325ull;
  for (size_t i = 0; i < n; i++) h = gxc::fnv1a_step(h, (uint8_t)s[i]);
  return h;
}
template <class T>
static int upload(gx_engine *e, const T *src, size_t n, const T **dst) {
  void *p = nullptr;
  size_t bytes = std::max<size_t>(sizeof(T) * n, 16);
  if (hipMalloc(&p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return GX_ENOMEM;
  }
  e->codec->owned.push_back(p);
  if (n) HIPCHK(hipMemcpy(p, src, sizeof(T) * n, hipMemcpyHostToDevice));
  *dst = (const T *)p;
  return GX_OK;
}

// ---------------------------------------------------------------------------------- scans --
// exclusive scan of exactly m elements in place (op order = element order)
template <class M, int ITEMS>
static int mscan(gx_engine *e, typename M::T *x, size_t m, char *scratch, size_t &soff) {
  typedef typename M::T T;
  const size_t per = 256 * ITEMS;
  const size_t nb = (m + per - 1) / per;
  soff = (soff + 255) & ~(size_t)255;
  T *tot = (T *)(scratch + soff);
  soff += sizeof(T) * (nb + 1);
  gxc::k_mscan_block<M, ITEMS><<<(unsigned)nb, 256, 0, e->stream>>>(x, m, tot);
  if (nb > 1) {
    int rc = mscan<M, ITEMS>(e, tot, nb, scratch, soff);
    if (rc) return rc;
    gxc::k_mscan_add<M, ITEMS><<<(unsigned)nb, 256, 0, e->stream>>>(x, m, tot);
  }
  HIPCHK(hipGetLastError());
  return GX_OK;
}
template <class M, int ITEMS>
static size_t mscan_scratch(size_t m) {
  size_t s = 0, per = 256 * ITEMS;
  while (true) {
    size_t nb = (m + per - 1) / per;
    s += 256 + sizeof(typename M::T) * (nb + 1);
    if (nb <= 1) break;
    m = nb;
  }
  return s;
}

// ------------------------------------------------------------------------------- encoder --
static int enc_impl(gx_engine *e, uint32_t view, char *out, uint64_t cap, uint64_t *n_out) {
  CodecState *c = e->codec;
  const Dev &d = e->d;
  const uint32_t vi = view - d.lo;
  void *base;
  const size_t sc = mscan_scratch<gxc::MAdd32, 16>(d.H + 1);
  int rc = dbuf(c->enc, 2 * (sizeof(uint32_t) * (d.H + 1) + 256) + sc, &base);
  if (rc) return rc;
  Bump bp;
  uint32_t *len = bp.take<uint32_t>((char *)base, d.H + 1);
  uint32_t *off = bp.take<uint32_t>((char *)base, d.H + 1);
  size_t soff = bp.off;
  int64_t vlc = 0;
  uint32_t tot = 0;
  {
    LaunchTimer t(e, GX_K_ENCODE);
    gxc::k_enc_len<<<nblk(d.H, 4), 256, 0, e->stream>>>(d, c->nm, vi, len);
    HIPCHK(hipMemcpyAsync(off, len, sizeof(uint32_t) * d.H, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(hipMemsetAsync(off + d.H, 0, sizeof(uint32_t), e->stream));
    rc = mscan<gxc::MAdd32, 16>(e, off, d.H + 1, (char *)base, soff);
    if (rc) return rc;
  }
  HIPCHK(hipMemcpyAsync(&tot, off + d.H, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&vlc, d.vlc + vi, sizeof(int64_t), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  const uint64_t total = gxc::enc_frame_len(c->nm, vlc, c->ehost_len[view]) + (tot ? tot - 1 : 0);
  if (n_out) *n_out = total;
  if (cap < total) return GX_OK;
  void *dout;
  rc = dbuf(c->out, total + 64, &dout);
  if (rc) return rc;
  {
    LaunchTimer t(e, GX_K_ENCODE);
    gxc::k_enc_frame<<<1, 64, 0, e->stream>>>(d, c->nm, vi, off, (char *)dout);
    gxc::k_enc_write<<<nblk(d.H, 4), 256, 0, e->stream>>>(d, c->nm, vi, len, off, (char *)dout);
  }
  rc = d2h_staged(e, c->pin2, out, (const char *)dout, total);
  if (rc) return rc;
  rc = sync_check(e);
  if (rc) return rc;
  // algorithmic bytes: the view row and server times read, every output byte written and (but
  // for formatted times) read once from a fragment
  e->host_bytes[GX_K_ENCODE] += 8ull * d.R + 16ull * d.H + 2 * total;
  e->host_units[GX_K_ENCODE] += total;
  return GX_OK;
}

// ------------------------------------------------------------------------------- decoder --
// Runs the parser; on success n_rec records sit in x.recs (document order).
static int dec_impl(gx_engine *e, const char *buf, uint64_t len, gx_decode_stats *ds, gxc::Dec &x, uint32_t &n_rec) {
  CodecState *c = e->codec;
  if (ds) {
    memset(ds, 0, sizeof(*ds));
    ds->bytes = len;
    ds->error_at = -1;
  }
  n_rec = 0;
  if (len == 0 || len >= 0xFFFFFF00ull) {
    if (ds) ds->error_at = 0;
    return GX_EINVAL;
  }
  memset(&x, 0, sizeof(x));
  x.n = (uint32_t)len;
  x.nc = (uint32_t)((len + GXC_CH - 1) / GXC_CH);
  const uint32_t nc = x.nc;
  void *inp;
  int rc = dbuf(c->in, len + 64, &inp);
  if (rc) return rc;
  x.s = (const uint8_t *)inp;
  x.epoch = e->d.epoch;
  // phase 1: chunk summaries and scans
  const size_t sc1 = mscan_scratch<gxc::MMap, 16>(nc + 1) + mscan_scratch<gxc::MTD, 8>(nc + 1) +
                     mscan_scratch<gxc::MLO, 1>(nc + 1);
  const size_t b1 = 16 * 256 + (size_t)(nc + 1) * (1 + 12 * 4 + sizeof(gxc::TD) + sizeof(gxc::LO16)) + sc1 + 64;
  void *p1;
  rc = dbuf(c->ph1, b1, &p1);
  if (rc) return rc;
  Bump bp;
  char *B1 = (char *)p1;
  x.cmap = bp.take<uint8_t>(B1, nc + 1);
  x.ctok = bp.take<uint32_t>(B1, 4ull * nc);
  x.cdd = bp.take<int32_t>(B1, 4ull * nc);
  x.cmn = bp.take<int32_t>(B1, 4ull * nc);
  x.ctd = bp.take<gxc::TD>(B1, nc + 1);
  x.clo = bp.take<gxc::LO16>(B1, nc + 1);
  x.err = bp.take<unsigned long long>(B1, 1);
  x.win_top = bp.take<uint32_t>(B1, 1);
  x.cnt = bp.take<uint32_t>(B1, 4);
  size_t soff = bp.off;
  const uint8_t idmap = gxc::MMap::id();
  const gxc::TD td0 = gxc::MTD::id();
  const gxc::LO16 lo0 = gxc::MLO::id();
  HIPCHK(hipMemcpyAsync(inp, buf, len, hipMemcpyHostToDevice, e->stream));
  LaunchTimer tm(e, GX_K_DECODE);
  HIPCHK(hipMemsetAsync(x.err, 0xFF, sizeof(unsigned long long), e->stream));
  HIPCHK(hipMemsetAsync(x.win_top, 0, sizeof(uint32_t), e->stream));
  HIPCHK(hipMemsetAsync(x.cnt, 0, sizeof(uint32_t) * 4, e->stream));
  gxc::k_dec_fsm<<<nblk(nc, GXC_BT), GXC_BT, 0, e->stream>>>(x);
  HIPCHK(hipMemcpyAsync(x.cmap + nc, &idmap, 1, hipMemcpyHostToDevice, e->stream));
  rc = mscan<gxc::MMap, 16>(e, x.cmap, nc + 1, B1, soff);
  if (rc) return rc;
  gxc::k_dec_sel<<<nblk(nc, 256), 256, 0, e->stream>>>(x);
  HIPCHK(hipMemcpyAsync(x.ctd + nc, &td0, sizeof(td0), hipMemcpyHostToDevice, e->stream));
  rc = mscan<gxc::MTD, 8>(e, x.ctd, nc + 1, B1, soff);
  if (rc) return rc;
  gxc::k_dec_levels<<<nblk(nc, GXC_BT), GXC_BT, 0, e->stream>>>(x);
  HIPCHK(hipMemcpyAsync(x.clo + nc, &lo0, sizeof(lo0), hipMemcpyHostToDevice, e->stream));
  rc = mscan<gxc::MLO, 1>(e, x.clo, nc + 1, B1, soff);
  if (rc) return rc;
  uint8_t fmap = 0;
  gxc::TD ftd;
  unsigned long long err = 0;
  HIPCHK(hipMemcpyAsync(&fmap, x.cmap + nc, 1, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&ftd, x.ctd + nc, sizeof(ftd), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&err, x.err, sizeof(err), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  const int fst = fmap & 3;  // lexer state after the last byte
  x.T = ftd.tok;
  if (ds) ds->tokens = x.T;
  if (err != ~0ull || ftd.depth != 0 || fst == gxc::ST_STR || fst == gxc::ST_ESC || x.T == 0) {
    if (ds) ds->error_at = err != ~0ull ? (int64_t)err : (int64_t)len;
    return GX_EINVAL;
  }
  // phase 2: tokens, grammar, kinds, fields
  const uint32_t T = x.T;
  uint32_t dsz = 1024;
  while (dsz < T / 2) dsz <<= 1;
  x.dmask = dsz - 1;
  const size_t sc2 = mscan_scratch<gxc::MAdd32, 16>(T + 1);
  const size_t b2 = 12 * 256 + (size_t)(T + 1) * (5 * 4 + 3) + (size_t)dsz * 4 + sc2;
  void *p2;
  rc = dbuf(c->ph2, b2, &p2);
  if (rc) return rc;
  Bump bq;
  char *B2 = (char *)p2;
  x.tpos = bq.take<uint32_t>(B2, T + 1);
  x.tpar = bq.take<uint32_t>(B2, T + 1);
  x.tmt = bq.take<uint32_t>(B2, T + 1);
  x.taux = bq.take<uint32_t>(B2, T + 1);
  x.sflag = bq.take<uint32_t>(B2, T + 1);
  x.tkind = bq.take<uint8_t>(B2, T + 1);
  x.tflag = bq.take<uint8_t>(B2, T + 1);
  x.tck = bq.take<uint8_t>(B2, T + 1);
  x.dset = bq.take<uint32_t>(B2, dsz);
  size_t soff2 = bq.off;
  HIPCHK(hipMemsetAsync(x.tmt, 0xFF, sizeof(uint32_t) * (T + 1), e->stream));
  HIPCHK(hipMemsetAsync(x.taux, 0, sizeof(uint32_t) * (T + 1), e->stream));
  HIPCHK(hipMemsetAsync(x.tflag, 0, T + 1, e->stream));
  HIPCHK(hipMemsetAsync(x.tck, gxc::K_ANY, T + 1, e->stream));
  HIPCHK(hipMemsetAsync(x.dset, 0, sizeof(uint32_t) * dsz, e->stream));
  gxc::k_dec_emit<<<nblk(nc, GXC_BT), GXC_BT, 0, e->stream>>>(x);
  gxc::k_dec_check<<<nblk(T, 256), 256, 0, e->stream>>>(x);
  gxc::k_dec_kind<<<nblk(T, 256), 256, 0, e->stream>>>(x);
  gxc::k_dec_member<<<nblk(T, 256), 256, 0, e->stream>>>(x);
  gxc::k_dec_svcflag<<<nblk(T + 1, 256), 256, 0, e->stream>>>(x);
  rc = mscan<gxc::MAdd32, 16>(e, x.sflag, T + 1, B2, soff2);
  if (rc) return rc;
  uint32_t n_svc = 0;
  HIPCHK(hipMemcpyAsync(&n_svc, x.sflag + T, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&err, x.err, sizeof(err), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  if (err != ~0ull) {
    if (ds) ds->error_at = (int64_t)err;
    return GX_EINVAL;
  }
  // phase 3: services -> records
  const size_t sc3 = mscan_scratch<gxc::MAdd32, 16>(n_svc + 1);
  const size_t b3 = 4 * 256 + (size_t)(n_svc + 1) * (4 + 4 + 2 * sizeof(grec)) + sc3;
  void *p3;
  rc = dbuf(c->ph3, b3, &p3);
  if (rc) return rc;
  Bump br;
  char *B3 = (char *)p3;
  x.slist = br.take<uint32_t>(B3, n_svc + 1);
  x.rflag = br.take<uint32_t>(B3, n_svc + 1);
  x.rtmp = br.take<grec>(B3, n_svc + 1);
  x.recs = br.take<grec>(B3, n_svc + 1);
  x.seen = c->seen;
  size_t soff3 = br.off;
  gxc::k_dec_svclist<<<nblk(T, 256), 256, 0, e->stream>>>(x);
  gxc::k_dec_svc<<<nblk(n_svc + 1, 256), 256, 0, e->stream>>>(x, c->nm, e->d.H, e->d.S, n_svc);
  rc = mscan<gxc::MAdd32, 16>(e, x.rflag, n_svc + 1, B3, soff3);
  if (rc) return rc;
  gxc::k_dec_recs<<<nblk(std::max(n_svc, 1u), 256), 256, 0, e->stream>>>(x, n_svc);
  uint32_t cnt[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(&n_rec, x.rflag + n_svc, sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(cnt, x.cnt, sizeof(cnt), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&err, x.err, sizeof(err), hipMemcpyDeviceToHost, e->stream));
  rc = sync_check(e);
  if (rc) return rc;
  if (n_rec) gxc::k_seen_clear<<<nblk(n_rec, 256), 256, 0, e->stream>>>(c->seen, x.recs, n_rec);
  HIPCHK(hipGetLastError());
  e->host_bytes[GX_K_DECODE] += len + 16ull * n_rec;  // input read once, records written
  e->host_units[GX_K_DECODE] += len;
  if (err != ~0ull) {
    if (ds) ds->error_at = (int64_t)err;
    n_rec = 0;
    return GX_EINVAL;
  }
  if (ds) {
    ds->services = n_svc;
    ds->records = n_rec;
    ds->unknown = cnt[1];
    ds->invalid = cnt[2];
  }
  return GX_OK;
}

extern "C" {

int gx_set_names(gx_engine *e, const gx_names *in) {
  if (!e || !in || !in->host_off || !in->id_off || !in->pre_off || !in->post_off) return GX_EINVAL;
  const uint32_t H = e->d.H, R = e->d.R, S = e->d.S;
  if (in->host_off[0] || in->id_off[0] || in->pre_off[0] || in->post_off[0]) return GX_EINVAL;
  if ((in->host_off[H] && !in->hosts) || (in->id_off[R] && !in->ids) || (in->pre_off[R] && !in->pre) ||
      (in->post_off[R] && !in->post) || (in->cluster_name_len && !in->cluster_name))
    return GX_EINVAL;
  for (uint32_t o = 0; o < H; o++)
    if (in->host_off[o + 1] < in->host_off[o]) return GX_EINVAL;
  for (uint32_t r = 0; r < R; r++) {
    if (in->id_off[r + 1] < in->id_off[r] || in->pre_off[r + 1] < in->pre_off[r] || in->post_off[r + 1] < in->post_off[r])
      return GX_EINVAL;
    if ((in->pre_off[r + 1] - in->pre_off[r]) + (in->post_off[r + 1] - in->post_off[r]) + 1 > 65535) return GX_EINVAL;
  }
  // map-key orders (encoding/json sorts keys bytewise); names must be unique per map
  auto hs = [&](uint32_t o) { return std::string(in->hosts + in->host_off[o], in->host_off[o + 1] - in->host_off[o]); };
  auto is = [&](uint32_t r) { return std::string(in->ids + in->id_off[r], in->id_off[r + 1] - in->id_off[r]); };
  std::vector<uint32_t> horder(H), sorder(R);
  for (uint32_t o = 0; o < H; o++) horder[o] = o;
  std::sort(horder.begin(), horder.end(), [&](uint32_t a, uint32_t b) { return hs(a) < hs(b); });
  for (uint32_t k = 1; k < H; k++)
    if (hs(horder[k - 1]) == hs(horder[k])) return GX_EINVAL;
  for (uint32_t o = 0; o < H; o++) {
    uint32_t *so = &sorder[(size_t)o * S];
    for (uint32_t j = 0; j < S; j++) so[j] = j;
    std::sort(so, so + S, [&](uint32_t a, uint32_t b) { return is(o * S + a) < is(o * S + b); });
    for (uint32_t j = 1; j < S; j++)
      if (is(o * S + so[j - 1]) == is(o * S + so[j])) return GX_EINVAL;
  }
  // encoded strings
  std::string eh, ei, ec;
  std::vector<uint64_t> eho(H + 1, 0), eio(R + 1, 0);
  std::vector<uint32_t> ehl(H);
  for (uint32_t o = 0; o < H; o++) {
    go_json_string(eh, in->hosts + in->host_off[o], in->host_off[o + 1] - in->host_off[o]);
    eho[o + 1] = eh.size();
    ehl[o] = (uint32_t)(eho[o + 1] - eho[o]);
  }
  for (uint32_t r = 0; r < R; r++) {
    go_json_string(ei, in->ids + in->id_off[r], in->id_off[r + 1] - in->id_off[r]);
    eio[r + 1] = ei.size();
  }
  go_json_string(ec, in->cluster_name, in->cluster_name_len);
  // lookup tables (open addressing, linear probing; index + 1)
  const uint32_t hsz = pow2_at_least(std::max(2 * H, 16u)), isz = pow2_at_least(std::max(2 * R, 16u));
  std::vector<uint32_t> hht(hsz, 0), iht(isz, 0);
  for (uint32_t o = 0; o < H; o++) {
    uint32_t s = (uint32_t)fnv1a(in->hosts + in->host_off[o], in->host_off[o + 1] - in->host_off[o]) & (hsz - 1);
    while (hht[s]) s = (s + 1) & (hsz - 1);
    hht[s] = o + 1;
  }
  for (uint32_t r = 0; r < R; r++) {
    uint64_t h = gxc::id_hash(fnv1a(in->ids + in->id_off[r], in->id_off[r + 1] - in->id_off[r]), r / S);
    uint32_t s = (uint32_t)h & (isz - 1);
    while (iht[s]) s = (s + 1) & (isz - 1);
    iht[s] = r + 1;
  }
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  codec_free(e);
  e->codec = new CodecState();
  CodecState *c = e->codec;
  gxc::Names &nm = c->nm;
  int rc = GX_OK;
#define UP(src, n, dst)                  \
  do {                                   \
    rc = upload(e, src, n, &dst);        \
    if (rc) {                            \
      codec_free(e);                     \
      return rc;                         \
    }                                    \
  } while (0)
  UP(eh.data(), eh.size(), nm.ehost);
  UP(eho.data(), eho.size(), nm.ehost_off);
  UP(ei.data(), ei.size(), nm.eid);
  UP(eio.data(), eio.size(), nm.eid_off);
  UP(in->pre, in->pre_off[R], nm.pre);
  UP(in->pre_off, (size_t)R + 1, nm.pre_off);
  UP(in->post, in->post_off[R], nm.post);
  UP(in->post_off, (size_t)R + 1, nm.post_off);
  UP(in->hosts, in->host_off[H], nm.host);
  UP(in->host_off, (size_t)H + 1, nm.host_off);
  UP(in->ids, in->id_off[R], nm.id);
  UP(in->id_off, (size_t)R + 1, nm.id_off);
  UP(horder.data(), horder.size(), nm.host_order);
  UP(sorder.data(), sorder.size(), nm.svc_order);
  UP(hht.data(), hht.size(), nm.host_ht);
  UP(iht.data(), iht.size(), nm.id_ht);
  UP(ec.data(), ec.size(), nm.ecluster);
#undef UP
  nm.host_mask = hsz - 1;
  nm.id_mask = isz - 1;
  nm.ecluster_len = (uint32_t)ec.size();
  c->ehost_len = ehl;
  if (hipMalloc((void **)&c->seen, sizeof(uint32_t) * R) != hipSuccess) {
    (void)hipGetLastError();
    codec_free(e);
    return GX_ENOMEM;
  }
  HIPCHK(hipMemset(c->seen, 0, sizeof(uint32_t) * R));
  // every record's static message bytes follow the names (packPacket lengths = codec lengths)
  std::vector<uint16_t> sb(R);
  for (uint32_t r = 0; r < R; r++)
    sb[r] = (uint16_t)((in->pre_off[r + 1] - in->pre_off[r]) + (in->post_off[r + 1] - in->post_off[r]) + 1);
  HIPCHK(hipMemcpy(e->d.sbytes, sb.data(), sizeof(uint16_t) * R, hipMemcpyHostToDevice));
  return GX_OK;
}

int gx_local_state_json(gx_engine *e, uint32_t view, char *out, uint64_t cap, uint64_t *n_out) {
  if (!e || !own(e, view) || (cap && !out)) return GX_EINVAL;
  if (!e->codec) return GX_ENOENT;
  HIPCHK(hipSetDevice(e->device));
  return enc_impl(e, view, out, cap, n_out);
}

int gx_decode_state_json(gx_engine *e, const char *buf, uint64_t len, gx_service *out, uint32_t cap,
                         uint32_t *n_out, gx_decode_stats *ds) {
  if (!e || (len && !buf) || (cap && !out)) return GX_EINVAL;
  if (!e->codec) return GX_ENOENT;
  HIPCHK(hipSetDevice(e->device));
  gxc::Dec x;
  uint32_t n = 0;
  int rc = dec_impl(e, buf, len, ds, x, n);
  if (n_out) *n_out = rc ? 0 : n;
  if (rc) return rc;
  uint32_t m = std::min(n, cap);
  if (m) {
    std::vector<grec> tmp(m);
    HIPCHK(hipMemcpyAsync(tmp.data(), x.recs, sizeof(grec) * m, hipMemcpyDeviceToHost, e->stream));
    rc = sync_check(e);
    if (rc) return rc;
    for (uint32_t i = 0; i < m; i++) to_svc(e, &tmp[i], &out[i]);
  }
  return GX_OK;
}

int gx_merge_remote_state_json(gx_engine *e, uint32_t view, const char *buf, uint64_t len, gx_decode_stats *ds) {
  if (!e || !own(e, view) || (len && !buf)) return GX_EINVAL;
  if (!e->codec) return GX_ENOENT;
  HIPCHK(hipSetDevice(e->device));
  gxc::Dec x;
  uint32_t n = 0;
  int rc = dec_impl(e, buf, len, ds, x, n);
  if (rc) return rc;
  // Merge: the decoded records as one remote row, merged in key order by the push-pull pass
  void *rowp;
  const Dev &d = e->d;
  rc = dbuf(e->codec->out, sizeof(uint64_t) * d.R, &rowp);
  if (rc) return rc;
  uint64_t *row = (uint64_t *)rowp;
  set_round_fields(e);
  const bool ev = !e->log_views.empty();
  {
    LaunchTimer t(e, GX_K_AE);
    gxc::k_row_fill<<<nblk(d.R, 256), 256, 0, e->stream>>>(row, d.R);
    if (n) gxc::k_row_scatter<<<nblk(n, 256), 256, 0, e->stream>>>(row, x.recs, n);
    if (d.R % 2 == 0 && !ev) k_merge_row<true, false><<<1, 256, 0, e->stream>>>(e->d, view, row);
    else if (d.R % 2 == 0) k_merge_row<true, true><<<1, 256, 0, e->stream>>>(e->d, view, row);
    else if (!ev) k_merge_row<false, false><<<1, 256, 0, e->stream>>>(e->d, view, row);
    else k_merge_row<false, true><<<1, 256, 0, e->stream>>>(e->d, view, row);
  }
  return sync_check(e);
}

}  // extern "C"
