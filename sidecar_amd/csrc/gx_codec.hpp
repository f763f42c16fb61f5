// gx_codec.hpp — full-state JSON codec of the sidecar-gx engine, gfx950.
//
// LocalState() / MergeRemoteState() of services_delegate.go:146-167 carry the whole catalog as
// ffjson JSON (catalog/services_state_ffjson.go:771-803, :334-375; service/service_ffjson.go:
// 370-436; Servers/Services maps through encoding/json). Both directions are byte work over HBM:
//
// Encoder (one view):
//   k_enc_len    one wave per server in hostname order; lanes = that host's services in ID order;
//                entry lengths from the packed slot words, wave-reduced to the server length
//   (scan)       exclusive prefix over servers -> byte offset of every server
//   k_enc_write  one wave per server writes its bytes: static fragments (key, pre, post) copied
//                by the 64 lanes together, times formatted in registers
//
// Decoder (a data-parallel JSON parser, no sequential pass over the document):
//   k_dec_fsm    256-byte chunk per thread: the lexer state machine (OUT, SCALAR, STRING, ESCAPE)
//                run from all 4 start states at once -> a state map + per-state token / depth counts
//   (scans)      compose the state maps (start state of each chunk), sum tokens and depth,
//                max-scan the last open bracket per nesting level
//   k_dec_emit   tokens with their parent container and bracket match, SoA
//   k_dec_check  RFC 8259 grammar as a pair rule on adjacent tokens + bracket types, strings and
//                scalars validated
//   k_dec_kind   container kinds (state, Servers map, Server, Services map, Service, Ports, Port)
//   k_dec_member typed fields per key token (ffjson type errors), last-wins winners, duplicate map
//                keys through a device hash set
//   k_dec_svc    one thread per Service object: its ID / Hostname / Updated / Status, names lookup
//                in device hash tables -> records in document order (compaction scans)
// Merge then scatters the records into a row and runs the push-pull merge pass (ae_pair) on it.
#pragma once

namespace gxc {

enum { K_TOP, K_SERVERS, K_SERVER, K_SERVICES, K_SERVICE, K_PORTS, K_PORT, K_ANY };
enum : uint8_t { T_OBJ = '{', T_OBJE = '}', T_ARR = '[', T_ARRE = ']', T_COL = ':', T_COM = ',', T_STR = 'S',
                 T_SCL = 'V' };
enum { SC_NULL = 1, SC_BOOL = 2, SC_INT = 3, SC_FLOAT = 4 };  // scalar classes (tflag)
enum { ST_OUT = 0, ST_SCL = 1, ST_STR = 2, ST_ESC = 3 };
#define GXC_CH 256
#define GXC_NONE 0xffffffffu
#define GXC_MAXD GX_JSON_MAX_DEPTH

// device tables set by gx_set_names
struct Names {
  const char *ehost;       // encoded hostnames (JSON strings with quotes)
  const uint64_t *ehost_off;
  const char *eid;         // encoded IDs
  const uint64_t *eid_off;
  const char *pre, *post;  // Service JSON fragments around Updated
  const uint64_t *pre_off, *post_off;
  const char *host, *id;   // raw names (decoder lookup)
  const uint64_t *host_off, *id_off;
  const uint32_t *host_order, *svc_order;
  const uint32_t *host_ht, *id_ht;  // open addressing: index + 1, 0 = empty
  uint32_t host_mask, id_mask;
  const char *ecluster;
  uint32_t ecluster_len;
};

// ------------------------------------------------------------------------ shared scalars --
GXHD uint64_t fnv1a_step(uint64_t h, uint8_t c) { return (h ^ c) * 0x100000001B3ull; }
GXHD uint64_t id_hash(uint64_t hid, uint32_t owner) { return hid ^ mix64(0xA24BAED4963EE407ull + owner); }

GXHD void civil_from_days(int64_t z, int64_t &y, int64_t &m, int64_t &d) {
  z += 719468;
  int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  int64_t doe = z - era * 146097;
  int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  int64_t mp = (5 * doy + 2) / 153;
  d = doy - (153 * mp + 2) / 5 + 1;
  m = mp < 10 ? mp + 3 : mp - 9;
  y = yoe + era * 400 + (m <= 2);
}
GXHD int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
  y -= m <= 2;
  int64_t era = (y >= 0 ? y : y - 399) / 400;
  int64_t yoe = y - era * 400;
  int64_t doy = (153 * (m > 2 ? m - 3 : m + 9) + 2) / 5 + d - 1;
  int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}
// time.Time.MarshalJSON (quoted RFC3339Nano, UTC) of ns >= 0 into t[32]; returns the length
GXHD uint32_t fmt_time(int64_t ns, char *t) {
  int64_t secs = ns / 1000000000ll, frac = ns % 1000000000ll;
  int64_t days = secs / 86400, rem = secs % 86400, y, m, d;
  civil_from_days(days, y, m, d);
  int64_t hh = rem / 3600, mi = rem / 60 % 60, ss = rem % 60;
  t[0] = '"';
  t[1] = (char)('0' + y / 1000 % 10);
  t[2] = (char)('0' + y / 100 % 10);
  t[3] = (char)('0' + y / 10 % 10);
  t[4] = (char)('0' + y % 10);
  t[5] = '-';
  t[6] = (char)('0' + m / 10);
  t[7] = (char)('0' + m % 10);
  t[8] = '-';
  t[9] = (char)('0' + d / 10);
  t[10] = (char)('0' + d % 10);
  t[11] = 'T';
  t[12] = (char)('0' + hh / 10);
  t[13] = (char)('0' + hh % 10);
  t[14] = ':';
  t[15] = (char)('0' + mi / 10);
  t[16] = (char)('0' + mi % 10);
  t[17] = ':';
  t[18] = (char)('0' + ss / 10);
  t[19] = (char)('0' + ss % 10);
  uint32_t k = 20;
  if (frac) {
    t[k++] = '.';
    int64_t div = 100000000;
    while (frac) {
      t[k++] = (char)('0' + frac / div);
      frac %= div;
      div /= 10;
    }
  }
  t[k++] = 'Z';
  t[k++] = '"';
  return k;
}
// The length depends on the fraction only, so slot times (epoch-relative, the epoch a whole
// number of seconds) and absolute times have the same length.
GXHD uint32_t time_len(int64_t ns) {
  int64_t frac = ns % 1000000000ll;
  if (!frac) return 22;
  uint32_t n = 9;
  while (frac % 10 == 0) {
    frac /= 10;
    n--;
  }
  return 23 + n;
}
// time.Parse(`"`+RFC3339+`"`) on the raw bytes between the quotes (gx_oracle_json.c parse_rfc3339)
GXHD int parse_rfc3339(const uint8_t *s, uint32_t n, int64_t &sec, int64_t &nsec) {
#define DIG(i) (s[i] >= '0' && s[i] <= '9')
#define NUM2(i) ((s[i] - '0') * 10 + (s[i + 1] - '0'))
  if (n < 20) return -1;
  if (!DIG(0) || !DIG(1) || !DIG(2) || !DIG(3) || s[4] != '-' || !DIG(5) || !DIG(6) || s[7] != '-' || !DIG(8) ||
      !DIG(9) || s[10] != 'T' || !DIG(11) || !DIG(12) || s[13] != ':' || !DIG(14) || !DIG(15) || s[16] != ':' ||
      !DIG(17) || !DIG(18))
    return -1;
  int64_t y = (s[0] - '0') * 1000 + (s[1] - '0') * 100 + (s[2] - '0') * 10 + (s[3] - '0');
  int64_t mo = NUM2(5), d = NUM2(8), hh = NUM2(11), mi = NUM2(14), ss = NUM2(17);
  uint32_t i = 19;
  int64_t frac = 0;
  if (i < n && s[i] == '.') {
    i++;
    uint32_t f0 = i;
    while (i < n && DIG(i)) {
      if (i - f0 < 9) frac = frac * 10 + (s[i] - '0');
      i++;
    }
    if (i == f0) return -1;
    for (uint32_t k = i - f0; k < 9; k++) frac *= 10;
  }
  int64_t off = 0;
  if (i < n && s[i] == 'Z') {
    i++;
  } else if (i + 6 <= n && (s[i] == '+' || s[i] == '-') && DIG(i + 1) && DIG(i + 2) && s[i + 3] == ':' && DIG(i + 4) &&
             DIG(i + 5)) {
    int64_t oh = NUM2(i + 1), om = NUM2(i + 4);
    if (oh > 23 || om > 59) return -1;
    off = (oh * 3600 + om * 60) * (s[i] == '-' ? -1 : 1);
    i += 6;
  } else {
    return -1;
  }
  if (i != n) return -1;
  const int mdays[13] = {0, 31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
  if (mo < 1 || mo > 12 || d < 1 || d > mdays[mo] || (mo == 2 && d == 29 && !leap) || hh > 23 || mi > 59 || ss > 59)
    return -1;
  sec = days_from_civil(y, mo, d) * 86400 + hh * 3600 + mi * 60 + ss - off;
  nsec = frac;
  return 0;
#undef DIG
#undef NUM2
}

// ------------------------------------------------------------- scans over a monoid (device) --
// op(a, b) = a followed by b; exclusive scan in place over n elements, x[n] receives the total.
struct MAdd32 {
  typedef uint32_t T;
  static GXHD T id() { return 0; }
  static GXHD T op(T a, T b) { return a + b; }
};
struct TD {
  uint32_t tok;
  int32_t depth;
};
struct MTD {
  typedef TD T;
  static GXHD T id() { return TD{0, 0}; }
  static GXHD T op(T a, T b) { return TD{a.tok + b.tok, a.depth + b.depth}; }
};
struct MMap {  // 4-state maps, 2 bits per start state: (a then b)[s] = b[a[s]]
  typedef uint8_t T;
  static GXHD T id() { return 0xE4; }
  static GXHD T op(T a, T b) {
    T r = 0;
    for (int s = 0; s < 4; s++) r |= (T)(((b >> (2 * ((a >> (2 * s)) & 3))) & 3) << (2 * s));
    return r;
  }
};
struct LO16 {
  uint32_t v[GXC_MAXD];
};
struct MLO {  // last open bracket (token index + 1) per nesting level
  typedef LO16 T;
  static GXHD T id() {
    T r;
    for (int i = 0; i < GXC_MAXD; i++) r.v[i] = 0;
    return r;
  }
  static GXHD T op(const T &a, const T &b) {
    T r;
    for (int i = 0; i < GXC_MAXD; i++) r.v[i] = b.v[i] > a.v[i] ? b.v[i] : a.v[i];
    return r;
  }
};

template <class M, int ITEMS>
__global__ __launch_bounds__(256) void k_mscan_block(typename M::T *x, size_t n, typename M::T *tot) {
  typedef typename M::T T;
  __shared__ T sh[256];
  const uint32_t t = threadIdx.x;
  size_t base = ((size_t)blockIdx.x * 256 + t) * ITEMS;
  T acc = M::id();
#pragma unroll
  for (int i = 0; i < ITEMS; i++)
    if (base + i < n) acc = M::op(acc, x[base + i]);
  sh[t] = acc;
  __syncthreads();
  for (uint32_t o = 1; o < 256; o <<= 1) {
    T y = t >= o ? sh[t - o] : M::id();
    __syncthreads();
    if (t >= o) sh[t] = M::op(y, sh[t]);
    __syncthreads();
  }
  T pre = t ? sh[t - 1] : M::id();
  if (t == 255) tot[blockIdx.x] = sh[255];
#pragma unroll
  for (int i = 0; i < ITEMS; i++)
    if (base + i < n) {
      T v = x[base + i];
      x[base + i] = pre;
      pre = M::op(pre, v);
    }
}
template <class M, int ITEMS>
__global__ __launch_bounds__(256) void k_mscan_add(typename M::T *x, size_t n, const typename M::T *pre) {
  size_t base = (size_t)blockIdx.x * 256 * ITEMS;
  const typename M::T p = pre[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < 256u * ITEMS; i += 256)
    if (base + i < n) x[base + i] = M::op(p, x[base + i]);
}
template <class M>
__global__ void k_mscan_total(typename M::T *x, size_t n, const typename M::T *tot) {
  x[n] = tot[0];
}

// ----------------------------------------------------------------------------- encoder --
GXD void wcopy(char *dst, const char *src, uint32_t n, uint32_t lane) {
  for (uint32_t i = lane; i < n; i += 64) dst[i] = src[i];
}
template <int N>
GXD void wlit(char *dst, const char (&lit)[N], uint32_t lane) {
  if (lane < N - 1) dst[lane] = lit[lane];
}
__constant__ const char L_HEAD[] = "{\"Servers\":{";
__constant__ const char L_NAME[] = ":{\"Name\":";
__constant__ const char L_SVCS[] = ",\"Services\":{";
__constant__ const char L_LU[] = "},\"LastUpdated\":";
__constant__ const char L_LC[] = ",\"LastChanged\":";
__constant__ const char L_TLC[] = "},\"LastChanged\":";
__constant__ const char L_CN[] = ",\"ClusterName\":";
__constant__ const char L_HN[] = ",\"Hostname\":";
#define LLEN(x) ((uint32_t)sizeof(x) - 1)

GXD uint32_t entry_len(const Names &nm, uint32_t r, uint64_t w) {
  return (uint32_t)(nm.eid_off[r + 1] - nm.eid_off[r]) + 1 + (uint32_t)(nm.pre_off[r + 1] - nm.pre_off[r]) +
         time_len(ts_of(w)) + (uint32_t)(nm.post_off[r + 1] - nm.post_off[r]) + 2;
}

// one wave per server position k (hostname order): srv_len[k] = its bytes + 1 separator, 0 if absent
__global__ __launch_bounds__(256) void k_enc_len(Dev d, Names nm, uint32_t vi, uint32_t *srv_len) {
  const uint32_t lane = threadIdx.x & 63, k = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= d.H) return;
  const uint32_t o = nm.host_order[k];
  const uint64_t *row = d.view + (size_t)vi * d.R;
  uint32_t len = 0;
  bool present = false;
  if (lane < d.S) {
    uint32_t r = o * d.S + nm.svc_order[(size_t)o * d.S + lane];
    uint64_t w = row[r];
    present = st_of(w) != GX_ABSENT;
    if (present) len = entry_len(nm, r, w);
  }
  uint32_t cnt = (uint32_t)__popcll(__ballot(present));
  for (int s = 32; s > 0; s >>= 1) len += __shfl_xor(len, s, 64);
  if (lane == 0) {
    uint32_t out = 0;
    if (cnt) {
      const gx_server_times &st = d.srvt[(size_t)vi * d.H + o];
      uint32_t eh = (uint32_t)(nm.ehost_off[o + 1] - nm.ehost_off[o]);
      out = eh + LLEN(L_NAME) + eh + LLEN(L_SVCS) + len + (cnt - 1) + LLEN(L_LU) + time_len(st.last_updated_ns) +
            LLEN(L_LC) + time_len(st.last_changed_ns) + 1 + 1;
    }
    srv_len[k] = out;
  }
}

// One wave per server. The server's bytes are assembled in a per-wave LDS buffer: the static
// fragments (ID key, pre, post) of each entry are copied by the 64 lanes together (coalesced
// reads); each entry's lane then formats its Updated time and Status in place; lane 0 writes the
// footer. The buffer starts at the output address mod 4, so the wave stores it with aligned
// dword stores (bytes only at the two ends). A server larger than the buffer is written by the
// same steps straight to the output.
#define ENC_LDS 12288
// server times and state.LastChanged: slot time -> absolute, 0 = never set (time.Unix(0, 0))
GXD int64_t abs_tm(const Dev &d, int64_t t) { return t ? t + d.epoch : 0; }
// Updated (Unix seconds + ns) -> slot time, clamped into the window like gx_ts_in (gx.h
// GX_TS_SHIFT): before it (pre-1970, zero time.Time) -> 0, stale for every lifespan; past it ->
// the window's end. The epoch is a whole number of seconds. (gx_oracle_json.c slot_time)
GXD int64_t slot_time(int64_t epoch, int64_t sec, int64_t nsec) {
  const int64_t es = epoch / GX_SEC_NS;
  if (sec < es) return 0;
  if (sec - es > GX_TS_LIMIT / GX_SEC_NS) return GX_TS_LIMIT - 1;
  const int64_t t = (sec - es) * GX_SEC_NS + nsec;
  return t >= GX_TS_LIMIT ? GX_TS_LIMIT - 1 : t;
}
GXD void put_bytes(char *dst, const char *src, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) dst[i] = src[i];
}
__global__ __launch_bounds__(256) void k_enc_write(Dev d, Names nm, uint32_t vi, const uint32_t *srv_len,
                                                   const uint32_t *srv_off, char *out) {
  __shared__ __attribute__((aligned(16))) char lds[4][ENC_LDS + 16];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6, k = blockIdx.x * 4 + wv;
  if (k >= d.H || srv_len[k] == 0) return;
  const uint32_t o = nm.host_order[k];
  const uint64_t gpos = LLEN(L_HEAD) + (uint64_t)srv_off[k];  // server's first byte in the output
  const uint32_t slen = srv_len[k] - ((srv_off[k] + srv_len[k] == srv_off[d.H]) ? 1u : 0u);  // + separator
  const bool in_lds = slen + 4 <= ENC_LDS;
  char *base = in_lds ? lds[wv] + (gpos & 3) : out + gpos;
  // this lane's entry (ID order)
  uint32_t r = 0, len = 0, kn = 0, pn = 0, qn = 0;
  uint64_t w = GX_SLOT_ABSENT, eo = 0, po = 0, qo = 0;
  bool present = false;
  if (lane < d.S) {
    r = o * d.S + nm.svc_order[(size_t)o * d.S + lane];
    w = d.view[(size_t)vi * d.R + r];
    present = st_of(w) != GX_ABSENT;
    if (present) {
      eo = nm.eid_off[r];
      kn = (uint32_t)(nm.eid_off[r + 1] - eo);
      po = nm.pre_off[r];
      pn = (uint32_t)(nm.pre_off[r + 1] - po);
      qo = nm.post_off[r];
      qn = (uint32_t)(nm.post_off[r + 1] - qo);
      len = kn + 1 + pn + time_len(ts_of(w)) + qn + 3;  // key : pre time post status } ,
    }
  }
  uint32_t inc = len;
  for (int s = 1; s < 64; s <<= 1) {
    uint32_t y = __shfl_up(inc, s, 64);
    if ((int)lane >= s) inc += y;
  }
  const uint32_t tot = __shfl(inc, 63, 64);
  const char *eh = nm.ehost + nm.ehost_off[o];
  const uint32_t ehn = (uint32_t)(nm.ehost_off[o + 1] - nm.ehost_off[o]);
  wcopy(base, eh, ehn, lane);
  wcopy(base + ehn, L_NAME, LLEN(L_NAME), lane);
  wcopy(base + ehn + LLEN(L_NAME), eh, ehn, lane);
  wcopy(base + 2 * ehn + LLEN(L_NAME), L_SVCS, LLEN(L_SVCS), lane);
  char *ent = base + 2 * ehn + LLEN(L_NAME) + LLEN(L_SVCS);
  // static fragments, entry by entry, all lanes copying
  const uint64_t pall = __ballot(present);
  uint64_t pm = pall;
  while (pm) {
    const int j = __ffsll((unsigned long long)pm) - 1;
    pm &= pm - 1;
    char *q = ent + (__shfl(inc, j, 64) - __shfl(len, j, 64));
    const uint32_t jk = __shfl(kn, j, 64), jp = __shfl(pn, j, 64), jq = __shfl(qn, j, 64);
    const uint32_t jt = time_len(ts_of(__shfl(w, j, 64)));
    wcopy(q, nm.eid + __shfl(eo, j, 64), jk, lane);
    wcopy(q + jk + 1, nm.pre + __shfl(po, j, 64), jp, lane);
    wcopy(q + jk + 1 + jp + jt, nm.post + __shfl(qo, j, 64), jq, lane);
  }
  if (present) {  // this lane's own entry: ':', Updated, Status, '}', ','
    char *q = ent + (inc - len);
    q[kn] = ':';
    q += kn + 1 + pn;
    q += fmt_time(ts_of(w) + d.epoch, q) + qn;
    q[0] = (char)('0' + st_of(w));
    q[1] = '}';
    if (pall >> (lane + 1)) q[2] = ',';  // not the last entry; the footer follows the last one
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane == 0) {
    char *f = ent + (tot ? tot - 1 : 0);
    const gx_server_times st = d.srvt[(size_t)vi * d.H + o];
    put_bytes(f, L_LU, LLEN(L_LU));
    f += LLEN(L_LU);
    f += fmt_time(abs_tm(d, st.last_updated_ns), f);
    put_bytes(f, L_LC, LLEN(L_LC));
    f += LLEN(L_LC);
    f += fmt_time(abs_tm(d, st.last_changed_ns), f);
    f[0] = '}';
    if (srv_off[k] + srv_len[k] != srv_off[d.H]) f[1] = ',';
  }
  if (!in_lds) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // LDS -> HBM: bytes up to the first 4-aligned output address, dwords, then the tail bytes
  const uint32_t head = (uint32_t)((4 - (gpos & 3)) & 3) < slen ? (uint32_t)((4 - (gpos & 3)) & 3) : slen;
  const uint32_t ndw = (slen - head) / 4, tail = slen - head - 4 * ndw;
  char *g = out + gpos;
  if (lane < head) g[lane] = base[lane];
  const uint32_t *ls = reinterpret_cast<const uint32_t *>(base + head);
  uint32_t *gd = reinterpret_cast<uint32_t *>(g + head);
  for (uint32_t i = lane; i < ndw; i += 64) gd[i] = ls[i];
  if (lane < tail) g[head + 4 * ndw + lane] = base[head + 4 * ndw + lane];
}

// header and tail of the state object (one wave)
__global__ void k_enc_frame(Dev d, Names nm, uint32_t vi, const uint32_t *srv_off, char *out) {
  const uint32_t lane = threadIdx.x;
  wcopy(out, L_HEAD, LLEN(L_HEAD), lane);
  uint32_t sb = srv_off[d.H];
  char *p = out + LLEN(L_HEAD) + (sb ? sb - 1 : 0);
  wcopy(p, L_TLC, LLEN(L_TLC), lane);
  p += LLEN(L_TLC);
  uint32_t tn = time_len(d.vlc[vi]);
  if (lane == 0) fmt_time(abs_tm(d, d.vlc[vi]), p);
  p += tn;
  wcopy(p, L_CN, LLEN(L_CN), lane);
  p += LLEN(L_CN);
  wcopy(p, nm.ecluster, nm.ecluster_len, lane);
  p += nm.ecluster_len;
  wcopy(p, L_HN, LLEN(L_HN), lane);
  p += LLEN(L_HN);
  const uint32_t v = d.lo + vi;
  const uint32_t ehn = (uint32_t)(nm.ehost_off[v + 1] - nm.ehost_off[v]);
  wcopy(p, nm.ehost + nm.ehost_off[v], ehn, lane);
  p += ehn;
  if (lane == 0) *p = '}';
}
GXHD uint64_t enc_frame_len(const Names &nm, int64_t vlc, uint32_t v_ehn) {
  return LLEN(L_HEAD) + LLEN(L_TLC) + time_len(vlc) + LLEN(L_CN) + nm.ecluster_len + LLEN(L_HN) + v_ehn + 1;
}

// ----------------------------------------------------------------------------- decoder --
struct Dec {
  int64_t epoch;     // the engine's (slot time 0)
  const uint8_t *s;  // input
  uint32_t n;        // input bytes
  uint32_t nc;       // chunks
  uint32_t T;        // tokens
  // per chunk
  uint8_t *cmap;     // state map (then: exclusive prefix)
  uint32_t *ctok;    // [4][nc] tokens per start state
  int32_t *cdd;      // [4][nc] depth delta per start state
  int32_t *cmn;      // [4][nc] min relative depth per start state
  TD *ctd;           // [nc + 1] (tokens, depth) of the chunk's start state, then exclusive prefix
  LO16 *clo;         // [nc + 1] last open per level inside the chunk, then exclusive max prefix
  // per token (SoA)
  uint32_t *tpos, *tpar, *tmt, *taux;
  uint8_t *tkind, *tflag, *tck;
  // services and records
  uint32_t *sflag;   // [T + 1] 1 = winning Service object (then: exclusive prefix = list index)
  uint32_t *slist;   // [n_svc] service open tokens, document order
  uint32_t *rflag;   // [n_svc + 1] 1 = emits a record (then: prefix)
  grec *rtmp;        // [n_svc] record of each service
  grec *recs;        // [n_rec] records in document order
  uint32_t *seen;    // [R] duplicate record keys
  uint32_t *dset;    // [dmask + 1] duplicate map keys (token + 1)
  uint32_t dmask;
  unsigned long long *err;  // first error offset (~0 = none)
  uint32_t *win_top;        // 1 + last "Servers" key token of the state object
  uint32_t *cnt;            // [4] services, unknown, invalid, dup
};

GXD void dec_err(const Dec &x, uint32_t pos) { atomicMin(x.err, (unsigned long long)pos); }
GXD bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
GXD bool is_struct(uint8_t c) { return c == '{' || c == '}' || c == '[' || c == ']' || c == ':' || c == ','; }

// the lexer step: state s, byte c -> new state; tok = a token starts at c
GXD int lex(int s, uint8_t c, bool &tok) {
  tok = false;
  if (s == ST_STR) return c == '"' ? ST_OUT : (c == '\\' ? ST_ESC : ST_STR);
  if (s == ST_ESC) return ST_STR;
  if (c == '"') {
    tok = true;
    return ST_STR;
  }
  if (is_struct(c)) {
    tok = true;
    return ST_OUT;
  }
  if (is_ws(c)) return ST_OUT;
  tok = s == ST_OUT;
  return ST_SCL;
}

// The byte-walking kernels stage their block's chunks in LDS first: 128 threads x 256 B, read
// from HBM with coalesced dword loads; chunk t sits at dword t * 65 (padded: the 128 walkers read
// 128 different banks). A walker reads a dword and steps through its 4 bytes.
#define GXC_BT 128
#define GXC_PAD 65
GXD void stage_chunks(const Dec &x, uint32_t *sb) {
  const uint32_t c0 = blockIdx.x * GXC_BT;
  const uint32_t *src = reinterpret_cast<const uint32_t *>(x.s) + (size_t)c0 * (GXC_CH / 4);
  const uint32_t ndw = (uint32_t)min((size_t)GXC_BT * (GXC_CH / 4), ((size_t)x.n + 3) / 4 - (size_t)c0 * (GXC_CH / 4));
  for (uint32_t i = threadIdx.x; i < ndw; i += GXC_BT) sb[(i >> 6) * GXC_PAD + (i & 63)] = src[i];
  __syncthreads();
}
#define WALK_BEGIN(a, b)                                            \
  for (uint32_t i0 = (a); i0 < (b); i0 += 4) {                      \
    const uint32_t dw = sb[threadIdx.x * GXC_PAD + ((i0 - (a)) >> 2)]; \
    for (uint32_t q = 0; q < 4 && i0 + q < (b); q++) {              \
      const uint32_t i = i0 + q;                                    \
      const uint8_t ch = (uint8_t)(dw >> (8 * q));
#define WALK_END \
  }              \
  }

// lexer transition table of one byte for the 4 states: byte 8*s = next state (bits 0-1), token
// starts (bit 2), opens a container (bit 3), closes one (bit 4)
GXD uint32_t lex_entry(uint32_t ch) {
  uint32_t w = 0;
  for (int s = 0; s < 4; s++) {
    bool tok;
    const bool was_out = s == ST_OUT || s == ST_SCL;
    const uint32_t ns = (uint32_t)lex(s, (uint8_t)ch, tok);
    const uint32_t op = was_out && (ch == '{' || ch == '['), cl = was_out && (ch == '}' || ch == ']');
    w |= (ns | (uint32_t)tok << 2 | op << 3 | cl << 4) << (8 * s);
  }
  return w;
}
__global__ __launch_bounds__(GXC_BT) void k_dec_fsm(Dec x) {
  __shared__ uint32_t sb[GXC_BT * GXC_PAD];
  __shared__ uint32_t ltab[256];
  for (uint32_t i = threadIdx.x; i < 256; i += GXC_BT) ltab[i] = lex_entry(i);
  stage_chunks(x, sb);
  const uint32_t c = blockIdx.x * GXC_BT + threadIdx.x;
  if (c >= x.nc) return;
  const uint32_t a = c * GXC_CH, b = min(a + GXC_CH, x.n);
  uint32_t st[4] = {0, 1, 2, 3};
  uint32_t tk[4] = {0, 0, 0, 0};
  int32_t dp[4] = {0, 0, 0, 0}, mn[4] = {0, 0, 0, 0};
  WALK_BEGIN(a, b)
  const uint32_t W = ltab[ch];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t e = (W >> (8 * st[k])) & 0x1Fu;
    st[k] = e & 3u;
    tk[k] += (e >> 2) & 1u;
    dp[k] += (int32_t)((e >> 3) & 1u) - (int32_t)((e >> 4) & 1u);
    mn[k] = min(mn[k], dp[k]);
  }
  (void)i;
  WALK_END
  uint8_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    m |= (uint8_t)(st[k] << (2 * k));
    x.ctok[k * x.nc + c] = tk[k];
    x.cdd[k * x.nc + c] = dp[k];
    x.cmn[k * x.nc + c] = mn[k];
  }
  x.cmap[c] = m;
}
// after the map scan: the chunk's start state selects its counts
__global__ __launch_bounds__(256) void k_dec_sel(Dec x) {
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= x.nc) return;
  const int s = x.cmap[c] & 3;  // prefix map applied to ST_OUT
  x.ctd[c] = TD{x.ctok[s * x.nc + c], x.cdd[s * x.nc + c]};
}
// depth never below zero; per chunk, the last open bracket (global token index + 1) per level
__global__ __launch_bounds__(GXC_BT) void k_dec_levels(Dec x) {
  __shared__ uint32_t sb[GXC_BT * GXC_PAD];
  __shared__ uint32_t ltab[256];
  for (uint32_t i = threadIdx.x; i < 256; i += GXC_BT) ltab[i] = lex_entry(i);
  stage_chunks(x, sb);
  const uint32_t c = blockIdx.x * GXC_BT + threadIdx.x;
  if (c >= x.nc) return;
  const int s0 = x.cmap[c] & 3;
  const TD td = x.ctd[c];
  if (td.depth + x.cmn[s0 * x.nc + c] < 0) dec_err(x, c * GXC_CH);
  LO16 lo = MLO::id();
  const uint32_t a = c * GXC_CH, b = min(a + GXC_CH, x.n);
  int s = s0;
  int32_t depth = td.depth;
  uint32_t ti = td.tok;
  WALK_BEGIN(a, b)
  const uint32_t e = (ltab[ch] >> (8 * s)) & 0x1Fu;
  s = (int)(e & 3u);
  if (e & 8u) {
    if (depth >= GXC_MAXD) dec_err(x, i);
    else {
#pragma unroll
      for (int L = 0; L < GXC_MAXD; L++)
        if (L == depth) lo.v[L] = ti + 1;
    }
    depth++;
  }
  if (e & 16u) depth--;
  ti += (e >> 2) & 1u;
  WALK_END
  x.clo[c] = lo;
}
// tokens (SoA): position, kind, level, parent container, bracket match
__global__ __launch_bounds__(GXC_BT) void k_dec_emit(Dec x) {
  __shared__ uint32_t sb[GXC_BT * GXC_PAD];
  __shared__ uint32_t sl[GXC_BT][GXC_MAXD + 1];
  __shared__ uint32_t ltab[256];
  for (uint32_t i = threadIdx.x; i < 256; i += GXC_BT) ltab[i] = lex_entry(i);
  stage_chunks(x, sb);
  const uint32_t c = blockIdx.x * GXC_BT + threadIdx.x;
  if (c >= x.nc) return;
  uint32_t *lo = sl[threadIdx.x];
  const LO16 pre = x.clo[c];
  for (int L = 0; L < GXC_MAXD; L++) lo[L] = pre.v[L];
  const uint32_t a = c * GXC_CH, b = min(a + GXC_CH, x.n);
  int s = x.cmap[c] & 3;
  int32_t depth = x.ctd[c].depth;
  uint32_t ti = x.ctd[c].tok;
  bool stop = false;
  WALK_BEGIN(a, b)
  const uint32_t e = (ltab[ch] >> (8 * s)) & 0x1Fu;
  s = (int)(e & 3u);
  if (!(e & 4u) || stop) continue;
  if (ti >= x.T) {  // cannot happen for a consistent scan; keeps writes in bounds
    stop = true;
    continue;
  }
  uint8_t kind = ch == '"' ? T_STR : (is_struct(ch) ? ch : T_SCL);
  uint32_t par = GXC_NONE, mt = GXC_NONE;
  if (kind == T_OBJ || kind == T_ARR) {
    if (depth > 0 && depth <= GXC_MAXD) par = lo[depth - 1] - 1;
    if (depth < GXC_MAXD) lo[depth] = ti + 1;
    depth++;
  } else if (kind == T_OBJE || kind == T_ARRE) {
    depth--;
    if (depth >= 0 && depth < GXC_MAXD) {
      mt = lo[depth] - 1;
      if (depth > 0) par = lo[depth - 1] - 1;
      if (mt != GXC_NONE) x.tmt[mt] = ti;
    }
    x.tmt[ti] = mt;
  } else if (depth > 0 && depth <= GXC_MAXD) {
    par = lo[depth - 1] - 1;
  }
  x.tpos[ti] = i;  // tflag, tck, taux are preset by the host (memset)
  x.tkind[ti] = kind;
  x.tpar[ti] = par;
  ti++;
  WALK_END
}

GXD int hexv(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
// end (index of the closing quote) of the string whose opening quote is at p; validates it
GXD uint32_t str_end(const Dec &x, uint32_t p, bool &ok) {
  uint32_t i = p + 1;
  ok = true;
  while (i < x.n) {
    const uint8_t c = x.s[i];
    if (c == '"') return i;
    if (c < 0x20) ok = false;
    if (c == '\\') {
      if (i + 1 >= x.n) {
        ok = false;
        return x.n;
      }
      const uint8_t e = x.s[i + 1];
      if (e == 'u') {
        if (i + 5 >= x.n || hexv(x.s[i + 2]) < 0 || hexv(x.s[i + 3]) < 0 || hexv(x.s[i + 4]) < 0 || hexv(x.s[i + 5]) < 0)
          ok = false;
        i += 6;
        continue;
      }
      if (!(e == '"' || e == '\\' || e == '/' || e == 'b' || e == 'f' || e == 'n' || e == 'r' || e == 't')) ok = false;
      i += 2;
      continue;
    }
    i++;
  }
  ok = false;
  return x.n;
}
// scalar class of the run at p (SC_*), 0 = invalid
GXD int scalar_class(const Dec &x, uint32_t p, uint32_t &end) {
  uint32_t i = p;
  while (i < x.n && !is_ws(x.s[i]) && !is_struct(x.s[i]) && x.s[i] != '"') i++;
  end = i;
  const uint8_t *s = x.s + p;
  const uint32_t n = i - p;
  if (n == 4 && s[0] == 'n' && s[1] == 'u' && s[2] == 'l' && s[3] == 'l') return SC_NULL;
  if (n == 4 && s[0] == 't' && s[1] == 'r' && s[2] == 'u' && s[3] == 'e') return SC_BOOL;
  if (n == 5 && s[0] == 'f' && s[1] == 'a' && s[2] == 'l' && s[3] == 's' && s[4] == 'e') return SC_BOOL;
  uint32_t k = 0;
  bool isint = true;
  if (k < n && s[k] == '-') k++;
  if (k < n && s[k] == '0') k++;
  else if (k < n && s[k] >= '1' && s[k] <= '9') {
    while (k < n && s[k] >= '0' && s[k] <= '9') k++;
  } else return 0;
  if (k < n && s[k] == '.') {
    isint = false;
    k++;
    uint32_t k0 = k;
    while (k < n && s[k] >= '0' && s[k] <= '9') k++;
    if (k == k0) return 0;
  }
  if (k < n && (s[k] == 'e' || s[k] == 'E')) {
    isint = false;
    k++;
    if (k < n && (s[k] == '+' || s[k] == '-')) k++;
    uint32_t k0 = k;
    while (k < n && s[k] >= '0' && s[k] <= '9') k++;
    if (k == k0) return 0;
  }
  if (k != n || n == 0) return 0;
  return isint ? SC_INT : SC_FLOAT;
}
GXD bool value_start(uint8_t k) { return k == T_STR || k == T_SCL || k == T_OBJ || k == T_ARR; }

// grammar: every adjacent token pair, bracket types, strings and scalars
__global__ __launch_bounds__(256) void k_dec_check(Dec x) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= x.T) return;
  const uint8_t a = x.tkind[t];
  const uint32_t pos = x.tpos[t];
  const uint32_t par = x.tpar[t];
  const uint8_t pk = par == GXC_NONE ? 0 : x.tkind[par];
  const bool last = t + 1 == x.T;
  const uint8_t b = last ? 0 : x.tkind[t + 1];
  bool ok = true;
  if (t == 0) ok = a == T_OBJ && x.tmt[0] == x.T - 1;
  if (par == GXC_NONE && t != 0 && !(last && a == T_OBJE)) ok = false;  // one top-level object only
  switch (a) {
    case T_OBJ: ok = ok && !last && (b == T_STR || b == T_OBJE); break;
    case T_ARR: ok = ok && !last && (value_start(b) || b == T_ARRE); break;
    case T_COL: ok = ok && pk == T_OBJ && !last && value_start(b); break;
    case T_COM:
      ok = ok && !last && (pk == T_OBJ ? b == T_STR : (pk == T_ARR && value_start(b)));
      break;
    case T_STR: {
      bool sok;
      str_end(x, pos, sok);
      ok = ok && sok;
      const uint8_t pv = t ? x.tkind[t - 1] : 0;
      const bool key = pk == T_OBJ && (pv == T_OBJ || pv == T_COM);
      if (key) ok = ok && !last && b == T_COL;
      else ok = ok && (last ? false : (b == T_COM || b == T_OBJE || b == T_ARRE));
      break;
    }
    case T_SCL: {
      uint32_t e;
      int sc = scalar_class(x, pos, e);
      ok = ok && sc != 0;
      x.tflag[t] = (uint8_t)sc;
      ok = ok && !last && (b == T_COM || b == T_OBJE || b == T_ARRE);
      break;
    }
    case T_OBJE:
    case T_ARRE: {
      const uint32_t m = x.tmt[t];
      ok = ok && m != GXC_NONE && m < x.T && x.tkind[m] == (a == T_OBJE ? T_OBJ : T_ARR);
      ok = ok && (last ? t == x.tmt[0] : (b == T_COM || b == T_OBJE || b == T_ARRE));
      break;
    }
    default: ok = false;
  }
  if (!ok) dec_err(x, pos);
}

// ---- strings: encoding/json unquote as a byte stream ----
struct Unq {
  const uint8_t *s;
  uint32_t i, end;
  uint8_t buf[4];
  uint32_t nb, bi;
};
GXHD uint32_t utf8_rune(const uint8_t *s, uint32_t n, uint32_t &sz) {
  const uint32_t c = s[0];
  if (c < 0x80) {
    sz = 1;
    return c;
  }
  if (c >= 0xC2 && c <= 0xDF && n >= 2 && (s[1] & 0xC0) == 0x80) {
    sz = 2;
    return ((c & 0x1Fu) << 6) | (s[1] & 0x3Fu);
  }
  if (c >= 0xE0 && c <= 0xEF && n >= 3 && (s[1] & 0xC0) == 0x80 && (s[2] & 0xC0) == 0x80) {
    uint32_t r = ((c & 0x0Fu) << 12) | ((s[1] & 0x3Fu) << 6) | (s[2] & 0x3Fu);
    if (r >= 0x800 && (r < 0xD800 || r > 0xDFFF)) {
      sz = 3;
      return r;
    }
  }
  if (c >= 0xF0 && c <= 0xF4 && n >= 4 && (s[1] & 0xC0) == 0x80 && (s[2] & 0xC0) == 0x80 && (s[3] & 0xC0) == 0x80) {
    uint32_t r = ((c & 0x07u) << 18) | ((s[1] & 0x3Fu) << 12) | ((s[2] & 0x3Fu) << 6) | (s[3] & 0x3Fu);
    if (r >= 0x10000 && r <= 0x10FFFF) {
      sz = 4;
      return r;
    }
  }
  sz = 1;
  return 0xFFFD;
}
GXD uint32_t utf8_put(uint8_t *o, uint32_t r) {
  if (r < 0x80) {
    o[0] = (uint8_t)r;
    return 1;
  }
  if (r < 0x800) {
    o[0] = (uint8_t)(0xC0 | (r >> 6));
    o[1] = (uint8_t)(0x80 | (r & 0x3F));
    return 2;
  }
  if (r < 0x10000) {
    o[0] = (uint8_t)(0xE0 | (r >> 12));
    o[1] = (uint8_t)(0x80 | ((r >> 6) & 0x3F));
    o[2] = (uint8_t)(0x80 | (r & 0x3F));
    return 3;
  }
  o[0] = (uint8_t)(0xF0 | (r >> 18));
  o[1] = (uint8_t)(0x80 | ((r >> 12) & 0x3F));
  o[2] = (uint8_t)(0x80 | ((r >> 6) & 0x3F));
  o[3] = (uint8_t)(0x80 | (r & 0x3F));
  return 4;
}
GXD uint32_t hex4(const uint8_t *s) {
  return (uint32_t)(hexv(s[0]) << 12 | hexv(s[1]) << 8 | hexv(s[2]) << 4 | hexv(s[3]));
}
// u.s/i/end over a validated string's content; returns the next unquoted byte or -1
GXD int unq_next(Unq &u) {
  if (u.bi < u.nb) return u.buf[u.bi++];
  if (u.i >= u.end) return -1;
  const uint8_t c = u.s[u.i];
  if (c == '\\') {
    const uint8_t e = u.s[u.i + 1];
    if (e == 'u') {
      uint32_t r = hex4(u.s + u.i + 2);
      u.i += 6;
      if (r >= 0xD800 && r < 0xE000) {
        uint32_t dec = 0xFFFD;
        if (r < 0xDC00 && u.i + 6 <= u.end && u.s[u.i] == '\\' && u.s[u.i + 1] == 'u' && hexv(u.s[u.i + 2]) >= 0 &&
            hexv(u.s[u.i + 3]) >= 0 && hexv(u.s[u.i + 4]) >= 0 && hexv(u.s[u.i + 5]) >= 0) {
          uint32_t r2 = hex4(u.s + u.i + 2);
          if (r2 >= 0xDC00 && r2 < 0xE000) {
            dec = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00);
            u.i += 6;
          }
        }
        r = dec;
      }
      u.nb = utf8_put(u.buf, r);
      u.bi = 1;
      return u.buf[0];
    }
    u.i += 2;
    return e == 'b' ? '\b' : e == 'f' ? '\f' : e == 'n' ? '\n' : e == 'r' ? '\r' : e == 't' ? '\t' : e;
  }
  if (c < 0x80) {
    u.i++;
    return c;
  }
  uint32_t sz;
  uint32_t r = utf8_rune(u.s + u.i, u.end - u.i, sz);
  if (r == 0xFFFD && sz == 1) {
    u.i += 1;
    u.nb = utf8_put(u.buf, 0xFFFD);
  } else {
    for (uint32_t k = 0; k < sz; k++) u.buf[k] = u.s[u.i + k];
    u.nb = sz;
    u.i += sz;
  }
  u.bi = 1;
  return u.buf[0];
}
GXD Unq unq_of(const Dec &x, uint32_t tok) {
  Unq u;
  u.s = x.s;
  u.i = x.tpos[tok] + 1;
  bool ok;
  u.end = str_end(x, x.tpos[tok], ok);
  u.nb = u.bi = 0;
  return u;
}
// ffjson key match: ASCII case-insensitive on the unquoted key
GXD bool key_is(const Dec &x, uint32_t tok, const char *name) {
  Unq u = unq_of(x, tok);
  for (uint32_t i = 0;; i++) {
    int c = unq_next(u);
    int m = (uint8_t)name[i];
    if (m == 0) return c < 0;
    if (c < 0) return false;
    if (c >= 'a' && c <= 'z') c -= 32;
    if (m >= 'a' && m <= 'z') m -= 32;
    if (c != m) return false;
  }
}
GXD bool unq_equal(const Dec &x, uint32_t ta, uint32_t tb) {
  Unq a = unq_of(x, ta), b = unq_of(x, tb);
  for (;;) {
    int ca = unq_next(a), cb = unq_next(b);
    if (ca != cb) return false;
    if (ca < 0) return true;
  }
}
GXD uint64_t unq_hash(const Dec &x, uint32_t tok, uint32_t &len) {
  Unq u = unq_of(x, tok);
  uint64_t h = 0xCBF29CE484222325ull;
  len = 0;
  for (int c; (c = unq_next(u)) >= 0; len++) h = fnv1a_step(h, (uint8_t)c);
  return h;
}
GXD bool unq_equal_raw(const Dec &x, uint32_t tok, const char *raw, uint32_t rn) {
  Unq u = unq_of(x, tok);
  for (uint32_t i = 0;; i++) {
    int c = unq_next(u);
    if (i == rn) return c < 0;
    if (c < 0 || (uint8_t)raw[i] != (uint32_t)c) return false;
  }
}

// Keys of at most 11 raw bytes without escapes (every field name) are packed, ASCII-uppercased,
// into two words and compared against packed constants; escaped keys take the unquoting path.
struct KP {
  uint64_t a, b;
  uint32_t len;  // 0xFE = escaped (slow path), 0xFD = longer than any field name
};
GXD KP key_pack(const Dec &x, uint32_t tok) {
  const uint32_t p = x.tpos[tok] + 1;
  KP k{0, 0, 0};
  for (uint32_t i = 0; i < 12; i++) {
    if (p + i >= x.n) {
      k.len = 0xFD;
      return k;
    }
    uint32_t c = x.s[p + i];
    if (c == '"') {
      k.len = i;
      return k;
    }
    if (c == '\\') {
      k.len = 0xFE;
      return k;
    }
    if (c >= 'a' && c <= 'z') c -= 32;
    if (i < 8) k.a |= (uint64_t)c << (8 * i);
    else k.b |= (uint64_t)c << (8 * (i - 8));
  }
  k.len = 0xFD;
  return k;
}
GXHD constexpr uint32_t cx_len(const char *s) {
  uint32_t n = 0;
  while (s[n]) n++;
  return n;
}
GXHD constexpr uint64_t cx_pack(const char *s, uint32_t from) {
  uint64_t v = 0;
  for (uint32_t i = 0; i < 8 && s[from + i]; i++) {
    uint32_t c = (uint8_t)s[from + i];
    if (c >= 'a' && c <= 'z') c -= 32;
    v |= (uint64_t)c << (8 * i);
  }
  return v;
}
#define KEQ(k, name) ((k).len == cx_len(name) && (k).a == cx_pack(name, 0) && (k).b == (cx_len(name) > 8 ? cx_pack(name, 8) : 0ull))

// fields (field ids per container kind)
enum { F_NONE, F_SERVERS, F_LASTCHANGED, F_CLUSTERNAME, F_HOSTNAME, F_NAME, F_SERVICES, F_LASTUPDATED, F_ID,
       F_IMAGE, F_PROXYMODE, F_CREATED, F_UPDATED, F_PORTS, F_STATUS, F_TYPE, F_IP, F_PORT, F_SERVICEPORT };
GXD int field_of_slow(const Dec &x, uint32_t key, int ck);
GXD int field_of(const Dec &x, uint32_t key, int ck) {
  const KP k = key_pack(x, key);
  if (k.len == 0xFE) return field_of_slow(x, key, ck);
  switch (ck) {
    case K_TOP:
      if (KEQ(k, "Servers")) return F_SERVERS;
      if (KEQ(k, "LastChanged")) return F_LASTCHANGED;
      if (KEQ(k, "ClusterName")) return F_CLUSTERNAME;
      if (KEQ(k, "Hostname")) return F_HOSTNAME;
      return F_NONE;
    case K_SERVER:
      if (KEQ(k, "Name")) return F_NAME;
      if (KEQ(k, "Services")) return F_SERVICES;
      if (KEQ(k, "LastUpdated")) return F_LASTUPDATED;
      if (KEQ(k, "LastChanged")) return F_LASTCHANGED;
      return F_NONE;
    case K_SERVICE:
      if (KEQ(k, "ID")) return F_ID;
      if (KEQ(k, "Name")) return F_NAME;
      if (KEQ(k, "Image")) return F_IMAGE;
      if (KEQ(k, "Created")) return F_CREATED;
      if (KEQ(k, "Hostname")) return F_HOSTNAME;
      if (KEQ(k, "Ports")) return F_PORTS;
      if (KEQ(k, "Updated")) return F_UPDATED;
      if (KEQ(k, "ProxyMode")) return F_PROXYMODE;
      if (KEQ(k, "Status")) return F_STATUS;
      return F_NONE;
    case K_PORT:
      if (KEQ(k, "Type")) return F_TYPE;
      if (KEQ(k, "Port")) return F_PORT;
      if (KEQ(k, "ServicePort")) return F_SERVICEPORT;
      if (KEQ(k, "IP")) return F_IP;
      return F_NONE;
  }
  return F_NONE;
}
GXD int field_of_slow(const Dec &x, uint32_t key, int ck) {
  switch (ck) {
    case K_TOP:
      if (key_is(x, key, "Servers")) return F_SERVERS;
      if (key_is(x, key, "LastChanged")) return F_LASTCHANGED;
      if (key_is(x, key, "ClusterName")) return F_CLUSTERNAME;
      if (key_is(x, key, "Hostname")) return F_HOSTNAME;
      return F_NONE;
    case K_SERVER:
      if (key_is(x, key, "Name")) return F_NAME;
      if (key_is(x, key, "Services")) return F_SERVICES;
      if (key_is(x, key, "LastUpdated")) return F_LASTUPDATED;
      if (key_is(x, key, "LastChanged")) return F_LASTCHANGED;
      return F_NONE;
    case K_SERVICE:
      if (key_is(x, key, "ID")) return F_ID;
      if (key_is(x, key, "Name")) return F_NAME;
      if (key_is(x, key, "Image")) return F_IMAGE;
      if (key_is(x, key, "Created")) return F_CREATED;
      if (key_is(x, key, "Hostname")) return F_HOSTNAME;
      if (key_is(x, key, "Ports")) return F_PORTS;
      if (key_is(x, key, "Updated")) return F_UPDATED;
      if (key_is(x, key, "ProxyMode")) return F_PROXYMODE;
      if (key_is(x, key, "Status")) return F_STATUS;
      return F_NONE;
    case K_PORT:
      if (key_is(x, key, "Type")) return F_TYPE;
      if (key_is(x, key, "Port")) return F_PORT;
      if (key_is(x, key, "ServicePort")) return F_SERVICEPORT;
      if (key_is(x, key, "IP")) return F_IP;
      return F_NONE;
  }
  return F_NONE;
}
// container kind of a child container of `pk` under field f (or array element)
GXD int child_kind(int pk, int f, uint8_t kind, bool &bad) {
  bad = false;
  const bool obj = kind == T_OBJ;
  switch (pk) {
    case K_TOP:
      if (f == F_SERVERS) { bad = !obj; return K_SERVERS; }
      bad = f != F_NONE;
      return K_ANY;
    case K_SERVERS: bad = !obj; return K_SERVER;
    case K_SERVER:
      if (f == F_SERVICES) { bad = !obj; return K_SERVICES; }
      bad = f != F_NONE;
      return K_ANY;
    case K_SERVICES: bad = !obj; return K_SERVICE;
    case K_SERVICE:
      if (f == F_PORTS) { bad = obj; return K_PORTS; }
      bad = f != F_NONE;
      return K_ANY;
    case K_PORTS: bad = !obj; return K_PORT;
    case K_PORT: bad = f != F_NONE; return K_ANY;
  }
  return K_ANY;
}
// container kinds: each open bracket walks its ancestor chain from the state object down
__global__ __launch_bounds__(256) void k_dec_kind(Dec x) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= x.T) return;
  const uint8_t k = x.tkind[t];
  if (k != T_OBJ && k != T_ARR) return;
  uint32_t chain[GXC_MAXD];
  int n = 0;
  for (uint32_t c = t; c != GXC_NONE && n < GXC_MAXD; c = x.tpar[c]) chain[n++] = c;
  int kind = K_TOP;
  bool bad = false;
  for (int i = n - 2; i >= 0; i--) {  // chain[n - 1] is the state object
    const uint32_t c = chain[i];
    int f = F_NONE;
    if (kind == K_ANY) break;
    if (c >= 2 && x.tkind[c - 1] == T_COL) {
      if (kind == K_TOP || kind == K_SERVER || kind == K_SERVICE || kind == K_PORT) f = field_of(x, c - 2, kind);
    }
    bool b;
    kind = child_kind(kind, f, x.tkind[c], b);
    bad = bad || (b && i == 0);  // each container reports its own type error
  }
  x.tck[t] = (uint8_t)kind;
  if (bad) dec_err(x, x.tpos[t]);
}

GXD bool int_value(const Dec &x, uint32_t tok, int64_t &v) {
  if (x.tkind[tok] != T_SCL || x.tflag[tok] != SC_INT) return false;
  const uint8_t *s = x.s + x.tpos[tok];
  uint32_t e;
  scalar_class(x, x.tpos[tok], e);
  const uint32_t n = e - x.tpos[tok];
  uint32_t k = 0;
  bool neg = false;
  if (s[0] == '-') {
    neg = true;
    k = 1;
  }
  const uint64_t lim = neg ? (1ull << 63) : (1ull << 63) - 1;
  uint64_t acc = 0;
  for (; k < n; k++) {
    const uint64_t dd = s[k] - '0';
    if (acc > (lim - dd) / 10) return false;
    acc = acc * 10 + dd;
  }
  v = neg ? (int64_t)(0 - acc) : (int64_t)acc;
  return true;
}
GXD bool is_null(const Dec &x, uint32_t v) { return x.tkind[v] == T_SCL && x.tflag[v] == SC_NULL; }
GXD bool time_ok(const Dec &x, uint32_t v, int64_t &sec, int64_t &nsec) {
  if (x.tkind[v] != T_STR) return false;
  bool ok;
  const uint32_t p = x.tpos[v], e = str_end(x, p, ok);
  return parse_rfc3339(x.s + p + 1, e - p - 1, sec, nsec) == 0;
}
// a duplicate key in one map (Servers or Services): device hash set keyed by (map, key)
GXD void map_key_insert(const Dec &x, uint32_t key, uint32_t map) {
  uint32_t len;
  const uint64_t h = mix64(unq_hash(x, key, len) ^ ((uint64_t)map << 1));
  for (uint32_t j = 0, slot = (uint32_t)h & x.dmask; j <= x.dmask; j++, slot = (slot + 1) & x.dmask) {
    const uint32_t prev = atomicCAS(&x.dset[slot], 0u, key + 1);
    if (prev == 0) return;
    const uint32_t other = prev - 1;
    if (x.tpar[other] == map && unq_equal(x, other, key)) {
      atomicAdd(&x.cnt[3], 1u);
      dec_err(x, x.tpos[key]);
      return;
    }
  }
}
// typed fields of every key (ffjson type errors), winners (last duplicate field), map keys
__global__ __launch_bounds__(256) void k_dec_member(Dec x) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= x.T) return;
  const uint32_t par = x.tpar[t];
  if (par == GXC_NONE) return;
  const int ck = x.tck[par];
  const uint8_t k = x.tkind[t];
  if (ck == K_PORTS && value_start(k) && (t == par + 1 || x.tkind[t - 1] == T_COM)) {  // []Port element
    if (!(k == T_OBJ || is_null(x, t))) dec_err(x, x.tpos[t]);
    return;
  }
  if (k != T_STR || t + 2 >= x.T || x.tkind[t + 1] != T_COL) return;
  const uint32_t v = t + 2;
  const uint8_t vk = x.tkind[v];
  const bool str_or_null = vk == T_STR || is_null(x, v);
  int64_t a, b;
  bool ok = true;
  if (ck == K_SERVERS || ck == K_SERVICES) {  // map: values are objects, keys unique
    ok = vk == T_OBJ;
    map_key_insert(x, t, par);
  } else if (ck == K_TOP || ck == K_SERVER || ck == K_SERVICE || ck == K_PORT) {
    switch (field_of(x, t, ck)) {
      case F_SERVERS:
        ok = vk == T_OBJ || is_null(x, v);
        atomicMax(x.win_top, t + 1);
        break;
      case F_SERVICES:
        ok = vk == T_OBJ || is_null(x, v);
        atomicMax(&x.taux[par], t + 1);
        break;
      case F_PORTS: ok = vk == T_ARR || is_null(x, v); break;
      case F_LASTCHANGED:
      case F_LASTUPDATED:
      case F_CREATED:
      case F_UPDATED: ok = is_null(x, v) || time_ok(x, v, a, b); break;
      case F_STATUS:
      case F_PORT:
      case F_SERVICEPORT: ok = is_null(x, v) || int_value(x, v, a); break;
      case F_NONE: break;
      default: ok = str_or_null;
    }
  }
  if (!ok) dec_err(x, x.tpos[v]);
}
// winning Service objects: under the last Services field of a Server in the last Servers field
__global__ __launch_bounds__(256) void k_dec_svcflag(Dec x) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t > x.T) return;
  uint32_t f = 0;
  if (t < x.T && x.tkind[t] == T_OBJ && x.tck[t] == K_SERVICE) {
    const uint32_t p = x.tpar[t], q = x.tpar[p], s = x.tpar[q];
    f = (p - 2 + 1 == x.taux[q] && s - 2 + 1 == *x.win_top) ? 1u : 0u;
  }
  x.sflag[t] = f;
}
__global__ __launch_bounds__(256) void k_dec_svclist(Dec x) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= x.T) return;
  if (x.sflag[t + 1] != x.sflag[t]) x.slist[x.sflag[t]] = t;
}
// one thread per winning Service: fields (last wins), names lookup, the record
__global__ __launch_bounds__(256) void k_dec_svc(Dec x, Names nm, uint32_t H, uint32_t S, uint32_t n_svc) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i > n_svc) return;
  if (i == n_svc) {
    x.rflag[i] = 0;
    return;
  }
  const uint32_t t = x.slist[i], end = x.tmt[t];
  uint32_t vid = GXC_NONE, vh = GXC_NONE, vu = GXC_NONE, vs = GXC_NONE;
  for (uint32_t m = t + 1; m < end;) {
    const uint32_t v = m + 2;
    switch (field_of(x, m, K_SERVICE)) {
      case F_ID: vid = v; break;
      case F_HOSTNAME: vh = v; break;
      case F_UPDATED: vu = v; break;
      case F_STATUS: vs = v; break;
    }
    const uint8_t vk = x.tkind[v];
    const uint32_t nx = (vk == T_OBJ || vk == T_ARR) ? x.tmt[v] + 1 : v + 1;
    if (nx < end && x.tkind[nx] == T_COM) m = nx + 1;
    else break;
  }
  uint32_t flag = 0;  // 1 = record, 2 = unknown, 3 = invalid
  grec g = {0, 0, 0};
  // names lookup (raw bytes, after unquoting); a null or missing string is ""
  uint32_t o = GXC_NONE, r = GXC_NONE;
  {
    uint32_t len = 0;
    uint64_t h = 0xCBF29CE484222325ull;
    if (vh != GXC_NONE && x.tkind[vh] == T_STR) h = unq_hash(x, vh, len);
    for (uint32_t j = 0, slot = (uint32_t)h & nm.host_mask; j <= nm.host_mask; j++, slot = (slot + 1) & nm.host_mask) {
      const uint32_t e = nm.host_ht[slot];
      if (!e) break;
      const uint32_t c = e - 1;
      const uint32_t cn = (uint32_t)(nm.host_off[c + 1] - nm.host_off[c]);
      bool eq = vh != GXC_NONE && x.tkind[vh] == T_STR ? unq_equal_raw(x, vh, nm.host + nm.host_off[c], cn) : cn == 0;
      if (eq) {
        o = c;
        break;
      }
    }
  }
  if (o != GXC_NONE) {
    uint32_t len = 0;
    uint64_t hid = 0xCBF29CE484222325ull;
    if (vid != GXC_NONE && x.tkind[vid] == T_STR) hid = unq_hash(x, vid, len);
    const uint64_t h = id_hash(hid, o);
    for (uint32_t j = 0, slot = (uint32_t)h & nm.id_mask; j <= nm.id_mask; j++, slot = (slot + 1) & nm.id_mask) {
      const uint32_t e = nm.id_ht[slot];
      if (!e) break;
      const uint32_t c = e - 1;
      if (c / S != o) continue;
      const uint32_t cn = (uint32_t)(nm.id_off[c + 1] - nm.id_off[c]);
      bool eq = vid != GXC_NONE && x.tkind[vid] == T_STR ? unq_equal_raw(x, vid, nm.id + nm.id_off[c], cn) : cn == 0;
      if (eq) {
        r = c;
        break;
      }
    }
  }
  if (r == GXC_NONE) {
    flag = 2;
  } else {
    int64_t sec = -62135596800ll, nsec = 0, st = 0;  // zero time.Time, zero Status
    if (vu != GXC_NONE && x.tkind[vu] == T_STR) time_ok(x, vu, sec, nsec);
    if (vs != GXC_NONE && x.tkind[vs] == T_SCL && x.tflag[vs] == SC_INT) int_value(x, vs, st);
    const bool bad = st < 0 || st > 6;
    flag = bad ? 3 : 1;
    g.w = pack(slot_time(x.epoch, sec, nsec), (int)st);
    g.r = r;
  }
  x.rtmp[i] = g;
  x.rflag[i] = flag == 1 ? 1u : 0u;
  if (flag == 2) atomicAdd(&x.cnt[1], 1u);
  if (flag == 3) atomicAdd(&x.cnt[2], 1u);
}
__global__ __launch_bounds__(256) void k_dec_recs(Dec x, uint32_t n_svc) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n_svc) return;
  if (x.rflag[i + 1] != x.rflag[i]) {
    const grec g = x.rtmp[i];
    x.recs[x.rflag[i]] = g;
    if (atomicAdd(&x.seen[g.r], 1u) != 0) {  // two records with one key
      atomicAdd(&x.cnt[3], 1u);
      dec_err(x, x.tpos[x.slist[i]]);
    }
  }
}
__global__ void k_row_fill(uint64_t *row, uint32_t R) {
  const uint32_t r = blockIdx.x * 256 + threadIdx.x;
  if (r < R) row[r] = GX_SLOT_ABSENT;
}
__global__ void k_row_scatter(uint64_t *row, const grec *recs, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) row[recs[i].r] = recs[i].w;
}
__global__ void k_seen_clear(uint32_t *seen, const grec *recs, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) seen[recs[i].r] = 0;
}

}  // namespace gxc

// MergeRemoteState's Merge of a decoded state: the push-pull pass with the decoded row as the
// remote row (key order, the model's Merge order; services_state.go:367-373)
template <bool VEC, bool EV>
__global__ __launch_bounds__(256) void k_merge_row(Dev d, uint32_t dst, const uint64_t *row) {
  __shared__ unsigned long long s_wave[4];
  __shared__ unsigned long long s_red[4];
  ae_pair<VEC, 1, false, EV>(d, dst, dst, false, s_wave, s_red, row, false);
}
