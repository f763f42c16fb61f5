/*
 * gx_oracle_json.c — CPU ORACLE of the full-state JSON codec. TEST INFRASTRUCTURE
 * ONLY; #included by gx_oracle.c (one translation unit).
 *
 * Restates, sequentially:
 *   LocalState()        services_delegate.go:146-151 -> ServicesState.Encode() services_state.go:117-125
 *                       -> ffjson MarshalJSONBuf (catalog/services_state_ffjson.go:771-803 ServicesState,
 *                       :334-375 Server, service/service_ffjson.go:370-436 Service), whose Servers and
 *                       Services maps fall back to encoding/json: keys sorted bytewise, strings
 *                       HTML-escaped, time.Time.MarshalJSON = quoted RFC3339Nano.
 *   MergeRemoteState()  services_delegate.go:153-167 -> catalog.Decode services_state.go:774-782
 *                       (ffjson UnmarshalJSON: typed fields, case-insensitive keys, last duplicate
 *                       field wins, unknown keys skipped) -> Merge :367-373 -> AddServiceEntry.
 * The parser is a plain recursive descent over a small DOM; the HIP engine's decoder is a
 * data-parallel tokenizer (sidecar_amd/csrc/gx_codec.hpp). Both follow the rules in include/gx.h.
 */

/* ------------------------------------------------------------------------- byte buffer -- */
typedef struct sbuf {
  char *p;
  size_t n, cap;
} sbuf;
static void sb_put(sbuf *b, const char *s, size_t n) {
  if (b->n + n > b->cap) {
    size_t c = b->cap ? b->cap : 256;
    while (c < b->n + n) c *= 2;
    b->p = (char *)realloc(b->p, c);
    b->cap = c;
  }
  memcpy(b->p + b->n, s, n);
  b->n += n;
}
static void sb_putc(sbuf *b, char c) { sb_put(b, &c, 1); }
static void sb_puts(sbuf *b, const char *s) { sb_put(b, s, strlen(s)); }

/* --------------------------------------------------------------------------- UTF-8 ------ */
/* utf8.DecodeRune: returns the rune and its size; invalid -> (0xFFFD, 1). */
static uint32_t utf8_rune(const unsigned char *s, size_t n, size_t *sz) {
  unsigned c = s[0];
  if (c < 0x80) { *sz = 1; return c; }
  if (c >= 0xC2 && c <= 0xDF && n >= 2 && (s[1] & 0xC0) == 0x80) {
    *sz = 2;
    return ((c & 0x1Fu) << 6) | (s[1] & 0x3Fu);
  }
  if (c >= 0xE0 && c <= 0xEF && n >= 3 && (s[1] & 0xC0) == 0x80 && (s[2] & 0xC0) == 0x80) {
    uint32_t r = ((c & 0x0Fu) << 12) | ((s[1] & 0x3Fu) << 6) | (s[2] & 0x3Fu);
    if (r >= 0x800 && (r < 0xD800 || r > 0xDFFF)) { *sz = 3; return r; }
  }
  if (c >= 0xF0 && c <= 0xF4 && n >= 4 && (s[1] & 0xC0) == 0x80 && (s[2] & 0xC0) == 0x80 && (s[3] & 0xC0) == 0x80) {
    uint32_t r = ((c & 0x07u) << 18) | ((s[1] & 0x3Fu) << 12) | ((s[2] & 0x3Fu) << 6) | (s[3] & 0x3Fu);
    if (r >= 0x10000 && r <= 0x10FFFF) { *sz = 4; return r; }
  }
  *sz = 1;
  return 0xFFFD;
}
static size_t utf8_put(unsigned char *o, uint32_t r) {
  if (r < 0x80) { o[0] = (unsigned char)r; return 1; }
  if (r < 0x800) { o[0] = (unsigned char)(0xC0 | (r >> 6)); o[1] = (unsigned char)(0x80 | (r & 0x3F)); return 2; }
  if (r < 0x10000) {
    o[0] = (unsigned char)(0xE0 | (r >> 12)); o[1] = (unsigned char)(0x80 | ((r >> 6) & 0x3F));
    o[2] = (unsigned char)(0x80 | (r & 0x3F));
    return 3;
  }
  o[0] = (unsigned char)(0xF0 | (r >> 18)); o[1] = (unsigned char)(0x80 | ((r >> 12) & 0x3F));
  o[2] = (unsigned char)(0x80 | ((r >> 6) & 0x3F)); o[3] = (unsigned char)(0x80 | (r & 0x3F));
  return 4;
}

/* encoding/json encodeState.string(s, escapeHTML=true) (Go 1.13, the module's CI toolchain). */
static void go_json_string(sbuf *b, const char *s0, size_t n) {
  static const char hex[] = "0123456789abcdef";
  const unsigned char *s = (const unsigned char *)s0;
  sb_putc(b, '"');
  size_t i = 0, start = 0;
  while (i < n) {
    unsigned c = s[i];
    if (c < 0x80) {
      if (c >= 0x20 && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&') { i++; continue; }
      sb_put(b, s0 + start, i - start);
      sb_putc(b, '\\');
      if (c == '"' || c == '\\') sb_putc(b, (char)c);
      else if (c == '\n') sb_putc(b, 'n');
      else if (c == '\r') sb_putc(b, 'r');
      else if (c == '\t') sb_putc(b, 't');
      else {
        char u[5] = {'u', '0', '0', hex[c >> 4], hex[c & 15]};
        sb_put(b, u, 5);
      }
      start = ++i;
      continue;
    }
    size_t sz;
    uint32_t r = utf8_rune(s + i, n - i, &sz);
    if ((r == 0xFFFD && sz == 1) || r == 0x2028 || r == 0x2029) {
      sb_put(b, s0 + start, i - start);
      sb_puts(b, r == 0xFFFD ? "\\ufffd" : (r == 0x2028 ? "\\u2028" : "\\u2029"));
      start = i + sz;
    }
    i += sz;
  }
  sb_put(b, s0 + start, n - start);
  sb_putc(b, '"');
}

/* ---------------------------------------------------------------- civil time (UTC) ------ */
static int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
  y -= m <= 2;
  int64_t era = (y >= 0 ? y : y - 399) / 400;
  int64_t yoe = y - era * 400;
  int64_t doy = (153 * (m > 2 ? m - 3 : m + 9) + 2) / 5 + d - 1;
  int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}
static void civil_from_days(int64_t z, int64_t *y, int64_t *m, int64_t *d) {
  z += 719468;
  int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  int64_t doe = z - era * 146097;
  int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  int64_t mp = (5 * doy + 2) / 153;
  *d = doy - (153 * mp + 2) / 5 + 1;
  *m = mp < 10 ? mp + 3 : mp - 9;
  *y = yoe + era * 400 + (*m <= 2);
}
/* time.Time.MarshalJSON of a UTC instant >= 0: "YYYY-MM-DDTHH:MM:SS[.frac]Z", quoted, fraction
 * with trailing zeros trimmed (RFC3339Nano). */
static void json_time(sbuf *b, int64_t ns) {
  int64_t secs = ns / 1000000000ll, frac = ns % 1000000000ll;
  int64_t days = secs / 86400, rem = secs % 86400, y, m, d;
  civil_from_days(days, &y, &m, &d);
  char t[48];
  int k = snprintf(t, sizeof t, "\"%04lld-%02lld-%02lldT%02lld:%02lld:%02lld", (long long)y, (long long)m,
                   (long long)d, (long long)(rem / 3600), (long long)(rem / 60 % 60), (long long)(rem % 60));
  if (frac) {
    char f[16];
    snprintf(f, sizeof f, ".%09lld", (long long)frac);
    int fl = 10;
    while (f[fl - 1] == '0') fl--;
    memcpy(t + k, f, (size_t)fl);
    k += fl;
  }
  t[k++] = 'Z';
  t[k++] = '"';
  sb_put(b, t, (size_t)k);
}
/* time.Parse(`"`+RFC3339+`"`, data) (time.Time.UnmarshalJSON, Go 1.13) on the raw bytes between
 * the quotes: YYYY-MM-DDTHH:MM:SS[.digits](Z|+hh:mm|-hh:mm). Returns 0 and the instant in
 * seconds + nanoseconds, or -1. */
static int parse_rfc3339(const unsigned char *s, size_t n, int64_t *sec, int64_t *nsec) {
#define DIG(i) (s[i] >= '0' && s[i] <= '9')
#define NUM2(i) ((s[i] - '0') * 10 + (s[i + 1] - '0'))
  if (n < 20) return -1;
  for (int i = 0; i < 4; i++)
    if (!DIG(i)) return -1;
  if (s[4] != '-' || !DIG(5) || !DIG(6) || s[7] != '-' || !DIG(8) || !DIG(9) || s[10] != 'T' || !DIG(11) ||
      !DIG(12) || s[13] != ':' || !DIG(14) || !DIG(15) || s[16] != ':' || !DIG(17) || !DIG(18))
    return -1;
  int64_t y = (s[0] - '0') * 1000 + (s[1] - '0') * 100 + (s[2] - '0') * 10 + (s[3] - '0');
  int64_t mo = NUM2(5), d = NUM2(8), hh = NUM2(11), mi = NUM2(14), ss = NUM2(17);
  size_t i = 19;
  int64_t frac = 0;
  if (i < n && s[i] == '.') {
    i++;
    size_t f0 = i;
    while (i < n && DIG(i)) {
      if (i - f0 < 9) frac = frac * 10 + (s[i] - '0');
      i++;
    }
    if (i == f0) return -1;
    for (size_t k = i - f0; k < 9; k++) frac *= 10;
  }
  int64_t off = 0;
  if (i < n && s[i] == 'Z') {
    i++;
  } else if (i + 6 <= n && (s[i] == '+' || s[i] == '-') && DIG(i + 1) && DIG(i + 2) && s[i + 3] == ':' &&
             DIG(i + 4) && DIG(i + 5)) {
    int64_t oh = NUM2(i + 1), om = NUM2(i + 4);
    if (oh > 23 || om > 59) return -1;
    off = (oh * 3600 + om * 60) * (s[i] == '-' ? -1 : 1);
    i += 6;
  } else {
    return -1;
  }
  if (i != n) return -1;
  static const int mdays[13] = {0, 31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  int leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
  if (mo < 1 || mo > 12 || d < 1 || d > mdays[mo] || (mo == 2 && d == 29 && !leap) || hh > 23 || mi > 59 ||
      ss > 59)
    return -1;
  *sec = days_from_civil(y, mo, d) * 86400 + hh * 3600 + mi * 60 + ss - off;
  *nsec = frac;
  return 0;
#undef DIG
#undef NUM2
}

/* ------------------------------------------------------------------------------ names -- */
typedef struct onames {
  char *cluster;
  uint64_t cluster_len;
  char *hosts, *ids, *pre, *post;
  uint64_t *host_off, *id_off, *pre_off, *post_off;
  sbuf ehost, eid, ecluster; /* encoded JSON strings */
  uint64_t *ehost_off, *eid_off;
  uint32_t *host_order; /* [H] hosts sorted by raw name (encoding/json map key order) */
  uint32_t *svc_order;  /* [R] per owner, services sorted by raw ID */
} onames;

static void free_names(gx_engine *e) {
  onames *nm = e->names;
  if (!nm) return;
  free(nm->cluster); free(nm->hosts); free(nm->ids); free(nm->pre); free(nm->post);
  free(nm->host_off); free(nm->id_off); free(nm->pre_off); free(nm->post_off);
  free(nm->ehost.p); free(nm->eid.p); free(nm->ecluster.p);
  free(nm->ehost_off); free(nm->eid_off); free(nm->host_order); free(nm->svc_order);
  free(nm);
  e->names = NULL;
}

static int bytes_cmp(const char *a, size_t na, const char *b, size_t nb) {
  size_t m = na < nb ? na : nb;
  int c = memcmp(a, b, m);
  return c ? c : (na < nb ? -1 : (na > nb ? 1 : 0));
}
static const onames *g_sort_names;
static uint32_t g_sort_owner;
static int cmp_host(const void *x, const void *y) {
  const onames *nm = g_sort_names;
  uint32_t a = *(const uint32_t *)x, b = *(const uint32_t *)y;
  return bytes_cmp(nm->hosts + nm->host_off[a], nm->host_off[a + 1] - nm->host_off[a], nm->hosts + nm->host_off[b],
                   nm->host_off[b + 1] - nm->host_off[b]);
}
static uint32_t g_sort_S;
static int cmp_svc(const void *x, const void *y) {
  const onames *nm = g_sort_names;
  uint64_t a = (uint64_t)g_sort_owner * g_sort_S + *(const uint32_t *)x;
  uint64_t b = (uint64_t)g_sort_owner * g_sort_S + *(const uint32_t *)y;
  return bytes_cmp(nm->ids + nm->id_off[a], nm->id_off[a + 1] - nm->id_off[a], nm->ids + nm->id_off[b],
                   nm->id_off[b + 1] - nm->id_off[b]);
}
static void *dup_bytes(const void *p, size_t n) {
  void *q = malloc(n ? n : 1);
  if (n) memcpy(q, p, n);
  return q;
}

int gx_set_names(gx_engine *e, const gx_names *in) {
  if (!e || !in || !in->host_off || !in->id_off || !in->pre_off || !in->post_off) return GX_EINVAL;
  uint32_t H = e->H, R = e->R, S = e->S;
  if (in->host_off[0] || in->id_off[0] || in->pre_off[0] || in->post_off[0]) return GX_EINVAL;
  for (uint32_t o = 0; o < H; o++)
    if (in->host_off[o + 1] < in->host_off[o]) return GX_EINVAL;
  for (uint32_t r = 0; r < R; r++) {
    if (in->id_off[r + 1] < in->id_off[r] || in->pre_off[r + 1] < in->pre_off[r] || in->post_off[r + 1] < in->post_off[r])
      return GX_EINVAL;
    if ((in->pre_off[r + 1] - in->pre_off[r]) + (in->post_off[r + 1] - in->post_off[r]) + 1 > 65535) return GX_EINVAL;
  }
  onames *nm = (onames *)calloc(1, sizeof(onames));
  nm->cluster = (char *)dup_bytes(in->cluster_name, in->cluster_name_len);
  nm->cluster_len = in->cluster_name_len;
  nm->hosts = (char *)dup_bytes(in->hosts, in->host_off[H]);
  nm->ids = (char *)dup_bytes(in->ids, in->id_off[R]);
  nm->pre = (char *)dup_bytes(in->pre, in->pre_off[R]);
  nm->post = (char *)dup_bytes(in->post, in->post_off[R]);
  nm->host_off = (uint64_t *)dup_bytes(in->host_off, sizeof(uint64_t) * (H + 1));
  nm->id_off = (uint64_t *)dup_bytes(in->id_off, sizeof(uint64_t) * (R + 1));
  nm->pre_off = (uint64_t *)dup_bytes(in->pre_off, sizeof(uint64_t) * (R + 1));
  nm->post_off = (uint64_t *)dup_bytes(in->post_off, sizeof(uint64_t) * (R + 1));
  nm->ehost_off = (uint64_t *)calloc(H + 1, sizeof(uint64_t));
  nm->eid_off = (uint64_t *)calloc(R + 1, sizeof(uint64_t));
  for (uint32_t o = 0; o < H; o++) {
    go_json_string(&nm->ehost, nm->hosts + nm->host_off[o], nm->host_off[o + 1] - nm->host_off[o]);
    nm->ehost_off[o + 1] = nm->ehost.n;
  }
  for (uint32_t r = 0; r < R; r++) {
    go_json_string(&nm->eid, nm->ids + nm->id_off[r], nm->id_off[r + 1] - nm->id_off[r]);
    nm->eid_off[r + 1] = nm->eid.n;
  }
  go_json_string(&nm->ecluster, nm->cluster, nm->cluster_len);
  nm->host_order = (uint32_t *)malloc(sizeof(uint32_t) * H);
  nm->svc_order = (uint32_t *)malloc(sizeof(uint32_t) * R);
  for (uint32_t o = 0; o < H; o++) nm->host_order[o] = o;
  g_sort_names = nm;
  g_sort_S = S;
  qsort(nm->host_order, H, sizeof(uint32_t), cmp_host);
  int dup = 0;
  for (uint32_t k = 1; k < H; k++) dup |= cmp_host(&nm->host_order[k - 1], &nm->host_order[k]) == 0;
  for (uint32_t o = 0; o < H && !dup; o++) {
    uint32_t *so = &nm->svc_order[(size_t)o * S];
    for (uint32_t j = 0; j < S; j++) so[j] = j;
    g_sort_owner = o;
    qsort(so, S, sizeof(uint32_t), cmp_svc);
    for (uint32_t j = 1; j < S; j++) dup |= cmp_svc(&so[j - 1], &so[j]) == 0;
  }
  if (dup) { /* hostnames and the IDs of one host must be unique (map keys) */
    e->names = nm;
    free_names(e);
    return GX_EINVAL;
  }
  free_names(e);
  e->names = nm;
  for (uint32_t r = 0; r < R; r++)
    e->sbytes[r] = (uint16_t)((nm->pre_off[r + 1] - nm->pre_off[r]) + (nm->post_off[r + 1] - nm->post_off[r]) + 1);
  return GX_OK;
}

/* ---------------------------------------------------------------------------- encoder -- */
int gx_local_state_json(gx_engine *e, uint32_t view, char *out, uint64_t cap, uint64_t *n_out) {
  if (!e || view < e->lo || view >= e->hi || (cap && !out)) return GX_EINVAL;
  const onames *nm = e->names;
  if (!nm) return GX_ENOENT;
  sbuf b = {0, 0, 0};
  const uint64_t *row = &e->view[(size_t)view * e->R];
  sb_puts(&b, "{\"Servers\":{");
  int first = 1;
  for (uint32_t k = 0; k < e->H; k++) {
    uint32_t o = nm->host_order[k];
    int any = 0;
    for (uint32_t j = 0; j < e->S; j++) any |= st_of(row[(size_t)o * e->S + j]) != GX_ABSENT;
    if (!any) continue; /* a server exists while it holds a record */
    if (!first) sb_putc(&b, ',');
    first = 0;
    const char *eh = nm->ehost.p + nm->ehost_off[o];
    size_t ehn = nm->ehost_off[o + 1] - nm->ehost_off[o];
    sb_put(&b, eh, ehn);
    sb_puts(&b, ":{\"Name\":");
    sb_put(&b, eh, ehn);
    sb_puts(&b, ",\"Services\":{");
    int fs = 1;
    for (uint32_t i = 0; i < e->S; i++) {
      uint32_t r = o * e->S + nm->svc_order[(size_t)o * e->S + i];
      uint64_t w = row[r];
      if (st_of(w) == GX_ABSENT) continue;
      if (!fs) sb_putc(&b, ',');
      fs = 0;
      sb_put(&b, nm->eid.p + nm->eid_off[r], nm->eid_off[r + 1] - nm->eid_off[r]);
      sb_putc(&b, ':');
      sb_put(&b, nm->pre + nm->pre_off[r], nm->pre_off[r + 1] - nm->pre_off[r]);
      json_time(&b, abs_ts(e, ts_of(w)));
      sb_put(&b, nm->post + nm->post_off[r], nm->post_off[r + 1] - nm->post_off[r]);
      sb_putc(&b, (char)('0' + st_of(w)));
      sb_putc(&b, '}');
    }
    const gx_server_times *st = &e->srvt[(size_t)view * e->H + o];
    sb_puts(&b, "},\"LastUpdated\":");
    json_time(&b, abs_tm(e, st->last_updated_ns));
    sb_puts(&b, ",\"LastChanged\":");
    json_time(&b, abs_tm(e, st->last_changed_ns));
    sb_putc(&b, '}');
  }
  sb_puts(&b, "},\"LastChanged\":");
  json_time(&b, abs_tm(e, e->vlc[view]));
  sb_puts(&b, ",\"ClusterName\":");
  sb_put(&b, nm->ecluster.p, nm->ecluster.n);
  sb_puts(&b, ",\"Hostname\":");
  sb_put(&b, nm->ehost.p + nm->ehost_off[view], nm->ehost_off[view + 1] - nm->ehost_off[view]);
  sb_putc(&b, '}');
  if (n_out) *n_out = b.n;
  if (cap >= b.n && b.n) memcpy(out, b.p, b.n);
  free(b.p);
  return GX_OK;
}

/* ---------------------------------------------------------------------------- decoder -- */
enum { JT_OBJ, JT_ARR, JT_STR, JT_NUM, JT_TRUE, JT_FALSE, JT_NULL };
typedef struct jnode {
  int type, is_int;
  size_t a, b;          /* value span: STR content between the quotes, NUM text */
  size_t ka, kb;        /* member key content span (object members) */
  int32_t first, next;  /* children list */
} jnode;
typedef struct jdoc {
  const unsigned char *s;
  size_t n, i;
  jnode *nd;
  size_t nn, ncap;
  uint64_t tokens;
  int64_t err;
} jdoc;

static void jerr(jdoc *d, size_t at) {
  if (d->err < 0) d->err = (int64_t)at;
}
static int32_t jnew(jdoc *d, int type) {
  if (d->nn == d->ncap) {
    d->ncap = d->ncap ? 2 * d->ncap : 1024;
    d->nd = (jnode *)realloc(d->nd, sizeof(jnode) * d->ncap);
  }
  jnode *x = &d->nd[d->nn];
  memset(x, 0, sizeof *x);
  x->type = type;
  x->first = x->next = -1;
  return (int32_t)d->nn++;
}
static void jws(jdoc *d) {
  while (d->i < d->n && (d->s[d->i] == ' ' || d->s[d->i] == '\t' || d->s[d->i] == '\n' || d->s[d->i] == '\r')) d->i++;
}
static int hexv(unsigned c) {
  if (c >= '0' && c <= '9') return (int)(c - '0');
  if (c >= 'a' && c <= 'f') return (int)(c - 'a' + 10);
  if (c >= 'A' && c <= 'F') return (int)(c - 'A' + 10);
  return -1;
}
/* a JSON string at d->i (the opening quote); content span -> [*a, *b) */
static int jstring(jdoc *d, size_t *a, size_t *b) {
  size_t i = d->i + 1;
  *a = i;
  while (i < d->n) {
    unsigned c = d->s[i];
    if (c == '"') {
      *b = i;
      d->i = i + 1;
      d->tokens++;
      return 0;
    }
    if (c < 0x20) { jerr(d, i); return -1; }
    if (c == '\\') {
      if (i + 1 >= d->n) { jerr(d, i); return -1; }
      unsigned x = d->s[i + 1];
      if (x == 'u') {
        if (i + 5 >= d->n || hexv(d->s[i + 2]) < 0 || hexv(d->s[i + 3]) < 0 || hexv(d->s[i + 4]) < 0 ||
            hexv(d->s[i + 5]) < 0) { jerr(d, i); return -1; }
        i += 6;
        continue;
      }
      if (!(x == '"' || x == '\\' || x == '/' || x == 'b' || x == 'f' || x == 'n' || x == 'r' || x == 't')) {
        jerr(d, i);
        return -1;
      }
      i += 2;
      continue;
    }
    i++;
  }
  jerr(d, d->i);
  return -1;
}
/* JSON number or literal at d->i: a maximal run of non-structural, non-space bytes. */
static int jscalar(jdoc *d, int32_t *out) {
  size_t a = d->i, i = a;
  while (i < d->n) {
    unsigned c = d->s[i];
    if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '{' || c == '}' || c == '[' || c == ']' || c == ':' ||
        c == ',' || c == '"')
      break;
    i++;
  }
  size_t n = i - a;
  const unsigned char *s = d->s + a;
  int type = -1, is_int = 0;
  if (n == 4 && !memcmp(s, "true", 4)) type = JT_TRUE;
  else if (n == 5 && !memcmp(s, "false", 5)) type = JT_FALSE;
  else if (n == 4 && !memcmp(s, "null", 4)) type = JT_NULL;
  else { /* -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)? */
    size_t k = 0;
    if (k < n && s[k] == '-') k++;
    if (k < n && s[k] == '0') k++;
    else if (k < n && s[k] >= '1' && s[k] <= '9') while (k < n && s[k] >= '0' && s[k] <= '9') k++;
    else k = n + 1;
    is_int = 1;
    if (k < n && s[k] == '.') {
      is_int = 0;
      k++;
      size_t k0 = k;
      while (k < n && s[k] >= '0' && s[k] <= '9') k++;
      if (k == k0) k = n + 1;
    }
    if (k < n && (s[k] == 'e' || s[k] == 'E')) {
      is_int = 0;
      k++;
      if (k < n && (s[k] == '+' || s[k] == '-')) k++;
      size_t k0 = k;
      while (k < n && s[k] >= '0' && s[k] <= '9') k++;
      if (k == k0) k = n + 1;
    }
    if (k == n && n) type = JT_NUM;
  }
  if (type < 0) { jerr(d, a); return -1; }
  int32_t x = jnew(d, type);
  d->nd[x].a = a;
  d->nd[x].b = i;
  d->nd[x].is_int = is_int;
  d->i = i;
  d->tokens++;
  *out = x;
  return 0;
}
static int jvalue(jdoc *d, int depth, int32_t *out) {
  jws(d);
  if (d->i >= d->n) { jerr(d, d->i); return -1; }
  unsigned c = d->s[d->i];
  if (c == '{' || c == '[') {
    if (depth >= GX_JSON_MAX_DEPTH) { jerr(d, d->i); return -1; }
    int obj = c == '{';
    int32_t x = jnew(d, obj ? JT_OBJ : JT_ARR), last = -1;
    d->i++;
    d->tokens++;
    jws(d);
    if (d->i < d->n && d->s[d->i] == (obj ? '}' : ']')) {
      d->i++;
      d->tokens++;
      *out = x;
      return 0;
    }
    for (;;) {
      size_t ka = 0, kb = 0;
      if (obj) {
        jws(d);
        if (d->i >= d->n || d->s[d->i] != '"') { jerr(d, d->i); return -1; }
        if (jstring(d, &ka, &kb)) return -1;
        jws(d);
        if (d->i >= d->n || d->s[d->i] != ':') { jerr(d, d->i); return -1; }
        d->i++;
        d->tokens++;
      }
      int32_t ch;
      if (jvalue(d, depth + 1, &ch)) return -1;
      d->nd[ch].ka = ka;
      d->nd[ch].kb = kb;
      if (last < 0) d->nd[x].first = ch;
      else d->nd[last].next = ch;
      last = ch;
      jws(d);
      if (d->i < d->n && d->s[d->i] == ',') {
        d->i++;
        d->tokens++;
        continue;
      }
      if (d->i < d->n && d->s[d->i] == (obj ? '}' : ']')) {
        d->i++;
        d->tokens++;
        break;
      }
      jerr(d, d->i);
      return -1;
    }
    *out = x;
    return 0;
  }
  if (c == '"') {
    int32_t x = jnew(d, JT_STR);
    size_t a, b;
    if (jstring(d, &a, &b)) return -1;
    d->nd[x].a = a;
    d->nd[x].b = b;
    *out = x;
    return 0;
  }
  return jscalar(d, out);
}

/* encoding/json unquote of a valid string's content [a, b) -> out (worst case 3x the input). */
static size_t junquote(const unsigned char *s, size_t a, size_t b, unsigned char *out) {
  size_t w = 0, i = a;
  while (i < b) {
    unsigned c = s[i];
    if (c == '\\') {
      unsigned x = s[i + 1];
      if (x == 'u') {
        uint32_t r = (uint32_t)(hexv(s[i + 2]) << 12 | hexv(s[i + 3]) << 8 | hexv(s[i + 4]) << 4 | hexv(s[i + 5]));
        i += 6;
        if (r >= 0xD800 && r < 0xE000) {
          uint32_t dec = 0xFFFD;
          if (r < 0xDC00 && i + 6 <= b && s[i] == '\\' && s[i + 1] == 'u' && hexv(s[i + 2]) >= 0 &&
              hexv(s[i + 3]) >= 0 && hexv(s[i + 4]) >= 0 && hexv(s[i + 5]) >= 0) {
            uint32_t r2 = (uint32_t)(hexv(s[i + 2]) << 12 | hexv(s[i + 3]) << 8 | hexv(s[i + 4]) << 4 | hexv(s[i + 5]));
            if (r2 >= 0xDC00 && r2 < 0xE000) {
              dec = 0x10000 + ((r - 0xD800) << 10) + (r2 - 0xDC00);
              i += 6;
            }
          }
          r = dec;
        }
        w += utf8_put(out + w, r);
        continue;
      }
      unsigned y = x == 'b' ? '\b' : x == 'f' ? '\f' : x == 'n' ? '\n' : x == 'r' ? '\r' : x == 't' ? '\t' : x;
      out[w++] = (unsigned char)y;
      i += 2;
      continue;
    }
    if (c < 0x80) {
      out[w++] = (unsigned char)c;
      i++;
      continue;
    }
    size_t sz;
    uint32_t r = utf8_rune(s + i, b - i, &sz);
    if (r == 0xFFFD && sz == 1) w += utf8_put(out + w, 0xFFFD);
    else {
      memcpy(out + w, s + i, sz);
      w += sz;
    }
    i += sz;
  }
  return w;
}
/* ffjson key match: exact or ASCII-case-insensitive on the unquoted key. */
static int key_is(const jdoc *d, const jnode *x, const char *name) {
  unsigned char buf[3 * 96 + 4];
  size_t kn = x->kb - x->ka;
  if (kn > 96) return 0; /* longer than any field name even with every byte \u-escaped */
  size_t n = junquote(d->s, x->ka, x->kb, buf);
  size_t m = strlen(name);
  if (n != m) return 0;
  for (size_t i = 0; i < n; i++) {
    unsigned a = buf[i], b = (unsigned char)name[i];
    if (a >= 'a' && a <= 'z') a -= 32;
    if (b >= 'a' && b <= 'z') b -= 32;
    if (a != b) return 0;
  }
  return 1;
}
static int is_str_or_null(const jnode *x) { return x->type == JT_STR || x->type == JT_NULL; }
static int is_time_or_null(const jdoc *d, const jnode *x) {
  if (x->type == JT_NULL) return 1;
  int64_t s, ns;
  return x->type == JT_STR && parse_rfc3339(d->s + x->a, x->b - x->a, &s, &ns) == 0;
}
/* strconv.ParseInt(text, 10, 64) of an integer token */
static int int_value(const jdoc *d, const jnode *x, int64_t *v) {
  if (x->type != JT_NUM || !x->is_int) return -1;
  const unsigned char *s = d->s + x->a;
  size_t n = x->b - x->a, k = 0;
  int neg = 0;
  if (s[0] == '-') { neg = 1; k = 1; }
  uint64_t acc = 0, lim = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
  for (; k < n; k++) {
    uint64_t dd = s[k] - '0';
    if (acc > (lim - dd) / 10) return -1;
    acc = acc * 10 + dd;
  }
  *v = neg ? (int64_t)(0 - acc) : (int64_t)acc;
  return 0;
}
static int is_int_or_null(const jdoc *d, const jnode *x) {
  int64_t v;
  return x->type == JT_NULL || int_value(d, x, &v) == 0;
}
/* two members of one map with the same unquoted key (sorted, adjacent compare) */
typedef struct jkey {
  unsigned char *p;
  size_t n;
} jkey;
static int cmp_jkey(const void *x, const void *y) {
  const jkey *a = (const jkey *)x, *b = (const jkey *)y;
  return bytes_cmp((const char *)a->p, a->n, (const char *)b->p, b->n);
}
static int dup_keys(const jdoc *d, const jnode *m) {
  size_t cnt = 0, bytes = 0;
  for (int32_t c = m->first; c >= 0; c = d->nd[c].next) {
    cnt++;
    bytes += 3 * (d->nd[c].kb - d->nd[c].ka) + 4;
  }
  if (cnt < 2) return 0;
  jkey *k = (jkey *)malloc(sizeof(jkey) * cnt);
  unsigned char *pool = (unsigned char *)malloc(bytes), *w = pool;
  size_t i = 0;
  for (int32_t c = m->first; c >= 0; c = d->nd[c].next, i++) {
    k[i].p = w;
    k[i].n = junquote(d->s, d->nd[c].ka, d->nd[c].kb, w);
    w += k[i].n;
  }
  qsort(k, cnt, sizeof(jkey), cmp_jkey);
  int rc = 0;
  for (i = 1; i < cnt && !rc; i++) rc = cmp_jkey(&k[i - 1], &k[i]) == 0;
  free(k);
  free(pool);
  return rc;
}

/* Updated (Unix seconds + ns) -> slot time, clamped into the engine's window like gx_ts_in
 * (gx.h GX_TS_SHIFT): before it (pre-1970, zero time.Time) -> 0, stale for every lifespan; past
 * it -> the window's end. The epoch is a whole number of seconds. */
static int64_t slot_time(const gx_engine *e, int64_t sec, int64_t nsec) {
  const int64_t es = e->epoch / GX_SEC_NS;
  if (sec < es) return 0;
  if (sec - es > GX_TS_LIMIT / GX_SEC_NS) return GX_TS_LIMIT - 1;
  const int64_t t = (sec - es) * GX_SEC_NS + nsec;
  return t >= GX_TS_LIMIT ? GX_TS_LIMIT - 1 : t;
}

typedef struct jrec {
  int64_t ns;     /* Updated as a slot time (slot_time) */
  uint32_t r;     /* record key */
  uint32_t st;
  uint64_t doc;   /* document order */
} jrec;
typedef struct jout {
  jrec *v;
  size_t n, cap;
  uint32_t services, unknown, invalid;
} jout;

static int find_host(const onames *nm, uint32_t H, const unsigned char *s, size_t n, uint32_t *o) {
  size_t lo = 0, hi = H;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    uint32_t x = nm->host_order[mid];
    int c = bytes_cmp(nm->hosts + nm->host_off[x], nm->host_off[x + 1] - nm->host_off[x], (const char *)s, n);
    if (c == 0) { *o = x; return 1; }
    if (c < 0) lo = mid + 1;
    else hi = mid;
  }
  return 0;
}
static int find_svc(const onames *nm, uint32_t S, uint32_t o, const unsigned char *s, size_t n, uint32_t *j) {
  size_t lo = 0, hi = S;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    uint64_t r = (uint64_t)o * S + nm->svc_order[(size_t)o * S + mid];
    int c = bytes_cmp(nm->ids + nm->id_off[r], nm->id_off[r + 1] - nm->id_off[r], (const char *)s, n);
    if (c == 0) { *j = nm->svc_order[(size_t)o * S + mid]; return 1; }
    if (c < 0) lo = mid + 1;
    else hi = mid;
  }
  return 0;
}

/* validate one Service object (service/service.go:32-42, Port :25-30); returns its fields */
static int j_service(const jdoc *d, const jnode *v, const jnode **id, const jnode **host, const jnode **upd,
                     const jnode **status) {
  *id = *host = *upd = *status = NULL;
  for (int32_t c = v->first; c >= 0; c = d->nd[c].next) {
    const jnode *x = &d->nd[c];
    if (key_is(d, x, "ID")) { if (!is_str_or_null(x)) return -1; *id = x; }
    else if (key_is(d, x, "Hostname")) { if (!is_str_or_null(x)) return -1; *host = x; }
    else if (key_is(d, x, "Name") || key_is(d, x, "Image") || key_is(d, x, "ProxyMode")) { if (!is_str_or_null(x)) return -1; }
    else if (key_is(d, x, "Updated")) { if (!is_time_or_null(d, x)) return -1; *upd = x; }
    else if (key_is(d, x, "Created")) { if (!is_time_or_null(d, x)) return -1; }
    else if (key_is(d, x, "Status")) { if (!is_int_or_null(d, x)) return -1; *status = x; }
    else if (key_is(d, x, "Ports")) {
      if (x->type == JT_NULL) continue;
      if (x->type != JT_ARR) return -1;
      for (int32_t p = x->first; p >= 0; p = d->nd[p].next) {
        const jnode *y = &d->nd[p];
        if (y->type == JT_NULL) continue;
        if (y->type != JT_OBJ) return -1;
        for (int32_t q = y->first; q >= 0; q = d->nd[q].next) {
          const jnode *z = &d->nd[q];
          if (key_is(d, z, "Type") || key_is(d, z, "IP")) { if (!is_str_or_null(z)) return -1; }
          else if (key_is(d, z, "Port") || key_is(d, z, "ServicePort")) { if (!is_int_or_null(d, z)) return -1; }
        }
      }
    }
  }
  return 0;
}

/* catalog.Decode + the record list Merge would apply. 0 = OK, else the document is rejected. */
static int j_decode(const gx_engine *e, jdoc *d, jout *out) {
  const onames *nm = e->names;
  int32_t top;
  jws(d);
  if (jvalue(d, 0, &top)) return -1;
  jws(d);
  if (d->i != d->n) { jerr(d, d->i); return -1; }
  const jnode *t = &d->nd[top];
  if (t->type != JT_OBJ) { jerr(d, 0); return -1; }
  const jnode *servers = NULL;
  int servers_set = 0;
  for (int32_t c = t->first; c >= 0; c = d->nd[c].next) { /* ServicesState fields */
    const jnode *x = &d->nd[c];
    if (key_is(d, x, "Servers")) {
      if (x->type == JT_NULL) { servers = NULL; servers_set = 1; continue; }
      if (x->type != JT_OBJ) { jerr(d, x->a); return -1; }
      servers = x;
      servers_set = 1;
      if (dup_keys(d, x)) { jerr(d, x->a); return -1; }
      for (int32_t s = x->first; s >= 0; s = d->nd[s].next) { /* Server values */
        const jnode *sv = &d->nd[s];
        if (sv->type != JT_OBJ) { jerr(d, sv->a); return -1; } /* null: Merge would panic */
        for (int32_t f = sv->first; f >= 0; f = d->nd[f].next) {
          const jnode *y = &d->nd[f];
          if (key_is(d, y, "Name")) { if (!is_str_or_null(y)) { jerr(d, y->a); return -1; } }
          else if (key_is(d, y, "LastUpdated") || key_is(d, y, "LastChanged")) { if (!is_time_or_null(d, y)) { jerr(d, y->a); return -1; } }
          else if (key_is(d, y, "Services")) {
            if (y->type == JT_NULL) continue;
            if (y->type != JT_OBJ || dup_keys(d, y)) { jerr(d, y->a); return -1; }
            for (int32_t q = y->first; q >= 0; q = d->nd[q].next) {
              const jnode *v = &d->nd[q], *a, *b, *u, *st;
              if (v->type != JT_OBJ || j_service(d, v, &a, &b, &u, &st)) { jerr(d, v->a); return -1; }
            }
          }
        }
      }
    } else if (key_is(d, x, "LastChanged")) {
      if (!is_time_or_null(d, x)) { jerr(d, x->a); return -1; }
    } else if (key_is(d, x, "ClusterName") || key_is(d, x, "Hostname")) {
      if (!is_str_or_null(x)) { jerr(d, x->a); return -1; }
    }
  }
  (void)servers_set;
  if (!servers) return 0;
  /* records of the winning Servers map, each server's winning Services map, document order */
  unsigned char *hb = NULL, *ib = NULL;
  uint64_t doc = 0;
  for (int32_t s = servers->first; s >= 0; s = d->nd[s].next) {
    const jnode *sv = &d->nd[s], *svcs = NULL;
    for (int32_t f = sv->first; f >= 0; f = d->nd[f].next)
      if (key_is(d, &d->nd[f], "Services")) svcs = d->nd[f].type == JT_OBJ ? &d->nd[f] : NULL;
    if (!svcs) continue;
    for (int32_t q = svcs->first; q >= 0; q = d->nd[q].next) {
      const jnode *v = &d->nd[q], *idn, *hn, *un, *stn;
      j_service(d, v, &idn, &hn, &un, &stn);
      out->services++;
      size_t nh = 0, ni = 0;
      if (hn && hn->type == JT_STR) {
        hb = (unsigned char *)realloc(hb, 3 * (hn->b - hn->a) + 4);
        nh = junquote(d->s, hn->a, hn->b, hb);
      }
      if (idn && idn->type == JT_STR) {
        ib = (unsigned char *)realloc(ib, 3 * (idn->b - idn->a) + 4);
        ni = junquote(d->s, idn->a, idn->b, ib);
      }
      uint32_t o, j;
      if (!find_host(nm, e->H, hb, nh, &o) || !find_svc(nm, e->S, o, ib, ni, &j)) {
        out->unknown++;
        continue;
      }
      int64_t sec = -62135596800ll, nsec = 0, stv = 0; /* zero time.Time, zero Status */
      if (un && un->type == JT_STR) parse_rfc3339(d->s + un->a, un->b - un->a, &sec, &nsec);
      if (stn && stn->type == JT_NUM) int_value(d, stn, &stv);
      const int bad = stv < 0 || stv > 6;
      const int64_t ns = slot_time(e, sec, nsec);
      if (bad) {
        out->invalid++;
        continue;
      }
      if (out->n == out->cap) {
        out->cap = out->cap ? 2 * out->cap : 256;
        out->v = (jrec *)realloc(out->v, sizeof(jrec) * out->cap);
      }
      jrec *rr = &out->v[out->n++];
      rr->ns = ns;
      rr->r = o * e->S + j;
      rr->st = (uint32_t)stv;
      rr->doc = doc++;
    }
  }
  free(hb);
  free(ib);
  /* two records with the same key: the reference order would be Go map order */
  uint8_t *seen = (uint8_t *)calloc(e->R, 1);
  int dupr = 0;
  for (size_t i = 0; i < out->n && !dupr; i++) {
    dupr = seen[out->v[i].r];
    seen[out->v[i].r] = 1;
  }
  free(seen);
  if (dupr) { jerr(d, 0); return -1; }
  return 0;
}

static int j_run(gx_engine *e, const char *buf, uint64_t len, jout *out, gx_decode_stats *ds) {
  jdoc d;
  memset(&d, 0, sizeof d);
  d.s = (const unsigned char *)buf;
  d.n = len;
  d.err = -1;
  memset(out, 0, sizeof *out);
  int rc = j_decode(e, &d, out);
  if (ds) {
    memset(ds, 0, sizeof *ds);
    ds->bytes = len;
    ds->tokens = d.tokens;
    ds->error_at = rc ? (d.err >= 0 ? d.err : 0) : -1;
    if (!rc) {
      ds->services = out->services;
      ds->records = (uint32_t)out->n;
      ds->unknown = out->unknown;
      ds->invalid = out->invalid;
    }
  }
  free(d.nd);
  return rc ? GX_EINVAL : GX_OK;
}

int gx_decode_state_json(gx_engine *e, const char *buf, uint64_t len, gx_service *out, uint32_t cap,
                         uint32_t *n_out, gx_decode_stats *ds) {
  if (!e || (len && !buf) || (cap && !out)) return GX_EINVAL;
  if (!e->names) return GX_ENOENT;
  jout o;
  int rc = j_run(e, buf, len, &o, ds);
  if (rc == GX_OK) {
    for (size_t i = 0; i < o.n && i < cap; i++) {
      out[i].updated_ns = abs_ts(e, o.v[i].ns);
      out[i].host = o.v[i].r / e->S;
      out[i].svc = (uint16_t)(o.v[i].r % e->S);
      out[i].status = (uint8_t)o.v[i].st;
      out[i].flags = 0;
    }
    if (n_out) *n_out = (uint32_t)o.n;
  } else if (n_out) {
    *n_out = 0;
  }
  free(o.v);
  return rc;
}

static int cmp_jrec_key(const void *x, const void *y) {
  uint32_t a = ((const jrec *)x)->r, b = ((const jrec *)y)->r;
  return a < b ? -1 : a > b;
}
int gx_merge_remote_state_json(gx_engine *e, uint32_t view, const char *buf, uint64_t len, gx_decode_stats *ds) {
  if (!e || view < e->lo || view >= e->hi || (len && !buf)) return GX_EINVAL;
  if (!e->names) return GX_ENOENT;
  jout o;
  int rc = j_run(e, buf, len, &o, ds);
  if (rc == GX_OK) {
    /* Merge in key order (the model's order for Merge, services_state.go:367-373) */
    qsort(o.v, o.n, sizeof(jrec), cmp_jrec_key);
    int64_t now = now_of(e);
    for (size_t i = 0; i < o.n; i++) {
      grec u = {pack(o.v[i].ns, (int)o.v[i].st), o.v[i].r, 0};
      add_entry(e, view, u, now, SRC_AE);
    }
    e->st.ae_slots += e->R; /* one full remote state, like gx_merge */
  }
  free(o.v);
  return rc;
}
