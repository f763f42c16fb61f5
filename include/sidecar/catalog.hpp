// sidecar/catalog.hpp — C++ host mirror of Sidecar's catalog API over the gx C-ABI (gx.h).
//
// Keeps the reference's method set and argument meaning so callers (and the parity tests in
// tests/cpp/) read like the reference:
//   catalog.ServicesState  (catalog/services_state.go:70-80)  -> sidecar::catalog::ServicesState
//   servicesDelegate       (services_delegate.go:20-27)       -> sidecar::ServicesDelegate
// Hostnames and service IDs are strings here, interned into the engine's (host, svc) indices by
// a Cluster. Error behaviour follows the reference: the hot path logs-and-continues (drops are
// counted by the engine, gx_stats); only misuse of this wrapper (an unknown hostname when the
// host table is full, a C-ABI error) throws std::runtime_error.
//
// Header-only; links against either implementation of gx.h (sidecar_amd/libgx.so, or the CPU
// oracle in tests).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <map>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../gx.h"

namespace sidecar {

// service.Service fields the merge path reads (service/service.go:32-42). Updated is UTC ns.
enum Status { ALIVE = GX_ALIVE, TOMBSTONE = GX_TOMBSTONE, UNHEALTHY = GX_UNHEALTHY, UNKNOWN = GX_UNKNOWN,
              DRAINING = GX_DRAINING };

struct Port {  // service.Port (service/service.go:25-30)
  std::string Type;
  int64_t Port = 0;
  int64_t ServicePort = 0;
  std::string IP;
};

struct Service {
  std::string ID;
  std::string Hostname;
  int64_t Updated = 0;
  int Status = ALIVE;
  // metadata the merge path does not read: ByService groups by Name; Encode() writes them all
  std::string Name;
  std::string Image;
  int64_t Created = 0;     // UTC ns
  std::vector<Port> Ports;
  std::string ProxyMode;
  bool IsTombstone() const { return Status == TOMBSTONE; }
  bool operator==(const Service &o) const {
    return ID == o.ID && Hostname == o.Hostname && Updated == o.Updated && Status == o.Status;  // the rest: metadata
  }
};

// ---- the reference's JSON for a Service (service/service_ffjson.go:370-436), as the engine's
// full-state codec needs it: the bytes before and after the Updated value (gx.h gx_names).
namespace json {
// encoding/json string encoding with HTML escaping (Go 1.13 encodeState.string, escapeHTML=true)
inline std::string quote(const std::string &in) {
  static const char *hex = "0123456789abcdef";
  std::string out = "\"";
  const unsigned char *b = reinterpret_cast<const unsigned char *>(in.data());
  const size_t n = in.size();
  for (size_t i = 0; i < n;) {
    const unsigned c = b[i];
    if (c < 0x80) {
      if (c >= 0x20 && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&') out += (char)c;
      else if (c == '"' || c == '\\') (out += '\\') += (char)c;
      else if (c == '\n') out += "\\n";
      else if (c == '\r') out += "\\r";
      else if (c == '\t') out += "\\t";
      else ((out += "\\u00") += hex[c >> 4]) += hex[c & 15];
      i++;
      continue;
    }
    // utf8.DecodeRune: an invalid sequence is one byte of U+FFFD
    uint32_t r = 0xFFFD, sz = 1;
    auto cont = [&](size_t k) { return i + k < n && (b[i + k] & 0xC0) == 0x80; };
    if (c >= 0xC2 && c <= 0xDF && cont(1)) {
      r = ((c & 0x1Fu) << 6) | (b[i + 1] & 0x3Fu);
      sz = 2;
    } else if (c >= 0xE0 && c <= 0xEF && cont(1) && cont(2)) {
      const uint32_t x = ((c & 0x0Fu) << 12) | ((b[i + 1] & 0x3Fu) << 6) | (b[i + 2] & 0x3Fu);
      if (x >= 0x800 && !(x >= 0xD800 && x <= 0xDFFF)) r = x, sz = 3;
    } else if (c >= 0xF0 && c <= 0xF4 && cont(1) && cont(2) && cont(3)) {
      const uint32_t x = ((c & 0x07u) << 18) | ((b[i + 1] & 0x3Fu) << 12) | ((b[i + 2] & 0x3Fu) << 6) | (b[i + 3] & 0x3Fu);
      if (x >= 0x10000 && x <= 0x10FFFF) r = x, sz = 4;
    }
    if (r == 0xFFFD && sz == 1) out += "\\ufffd";
    else if (r == 0x2028) out += "\\u2028";
    else if (r == 0x2029) out += "\\u2029";
    else out.append(in, i, sz);
    i += sz;
  }
  return out + "\"";
}
// time.Time.MarshalJSON of a UTC instant: quoted RFC3339Nano, fraction without trailing zeros
inline std::string time(int64_t ns) {
  int64_t secs = ns / 1000000000, frac = ns % 1000000000;
  if (frac < 0) frac += 1000000000, secs--;
  int64_t days = secs / 86400, rem = secs % 86400;
  if (rem < 0) rem += 86400, days--;
  // civil_from_days (proleptic Gregorian)
  const int64_t z = days + 719468, era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097, yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100), mp = (5 * doy + 2) / 153;
  const int64_t d = doy - (153 * mp + 2) / 5 + 1, m = mp < 10 ? mp + 3 : mp - 9, y = yoe + era * 400 + (m <= 2);
  char buf[64];
  std::snprintf(buf, sizeof buf, "%04lld-%02lld-%02lldT%02lld:%02lld:%02lld", (long long)y, (long long)m, (long long)d,
                (long long)(rem / 3600), (long long)(rem / 60 % 60), (long long)(rem % 60));
  std::string s = std::string("\"") + buf;
  if (frac) {
    char f[16];
    std::snprintf(f, sizeof f, ".%09lld", (long long)frac);
    std::string fs = f;
    while (fs.back() == '0') fs.pop_back();
    s += fs;
  }
  return s + "Z\"";
}
// (pre, post) of svc's JSON around its Updated value: {"ID":..,"Name":..,"Image":..,"Created":..,
// "Hostname":..,"Ports":..,"Updated":  and  ,"ProxyMode":..,"Status":
inline std::pair<std::string, std::string> fragments(const Service &svc) {
  std::string ports = "null";
  if (!svc.Ports.empty()) {
    ports = "[";
    for (size_t i = 0; i < svc.Ports.size(); i++) {
      const Port &p = svc.Ports[i];
      if (i) ports += ",";
      ports += "{\"Type\":" + quote(p.Type) + ",\"Port\":" + std::to_string(p.Port) + ",\"ServicePort\":" +
               std::to_string(p.ServicePort) + ",\"IP\":" + quote(p.IP) + "}";
    }
    ports += "]";
  }
  std::string pre = "{\"ID\":" + quote(svc.ID) + ",\"Name\":" + quote(svc.Name) + ",\"Image\":" + quote(svc.Image) +
                    ",\"Created\":" + time(svc.Created) + ",\"Hostname\":" + quote(svc.Hostname) + ",\"Ports\":" +
                    ports + ",\"Updated\":";
  std::string post = ",\"ProxyMode\":" + quote(svc.ProxyMode) + ",\"Status\":";
  return {pre, post};
}
}  // namespace json

// catalog.ChangeEvent (services_state.go:38-43)
struct ChangeEvent {
  Service Svc;
  int PreviousStatus = UNKNOWN;
  int64_t Time = 0;
};

// Server.LastUpdated / LastChanged (services_state.go:49-54); 0 = time.Unix(0, 0)
struct ServerTimes {
  int64_t LastUpdated = 0;
  int64_t LastChanged = 0;
};

inline void check(int rc, const char *what) {
  if (rc != GX_OK) throw std::runtime_error(std::string(what) + " failed: " + std::to_string(rc));
}

// One gx engine plus the string <-> index tables. Each host of the cluster has its own
// ServicesState view (a real Sidecar node has exactly one).
class Cluster {
 public:
  explicit Cluster(gx_params p) : p_(p) { check(gx_create(&p_, &e_), "gx_create"); }
  static gx_params Defaults(uint32_t hosts, uint32_t services_per_host) {
    gx_params p;
    gx_params_default(&p);
    p.n_hosts = hosts;
    p.n_services = services_per_host;
    return p;
  }
  ~Cluster() {
    if (e_) gx_destroy(e_);
  }
  Cluster(const Cluster &) = delete;
  Cluster &operator=(const Cluster &) = delete;

  gx_engine *engine() const { return e_; }
  const gx_params &params() const { return p_; }
  int64_t Now() const {
    int64_t r = 0;
    gx_get_round(e_, &r);
    return p_.t0_ns + r * p_.round_ns;
  }
  // Let simulated time pass (the reference reads time.Now(); the engine's clock is rounds).
  void Advance(int64_t rounds) {
    int64_t r = 0;
    check(gx_get_round(e_, &r), "gx_get_round");
    check(gx_set_round(e_, r + rounds), "gx_set_round");
  }
  void RunRounds(uint32_t n) { check(gx_run_rounds(e_, n), "gx_run_rounds"); }

  uint32_t Host(const std::string &name) {
    auto it = hosts_.find(name);
    if (it != hosts_.end()) return it->second;
    if (host_names_.size() >= p_.n_hosts) throw std::runtime_error("host table full: " + name);
    uint32_t id = (uint32_t)host_names_.size();
    hosts_[name] = id;
    host_names_.push_back(name);
    ids_.emplace_back();
    id_names_.emplace_back();
    slot_free_since_.emplace_back();
    return id;
  }
  // A service ID seen for the first time takes the owner's next free slot (the reference creates
  // it, services_state.go:310-318). When all S are taken, a slot that no view holds any more
  // (garbage-collected everywhere after TOMBSTONE_LIFESPAN, :645-653) is reused, but only once no
  // copy of its old record can still be merged anywhere. Every copy in a queue or in flight
  // carries the Updated of a stored version (+ at most 9 SendServices passes of 50 ns), and a
  // view collects a tombstone only once Updated < now - TOMBSTONE_LIFESPAN; IsStale drops a copy
  // once Updated < now - TOMBSTONE_LIFESPAN - 1 min (service.go:68-71). So when a slot is first
  // seen unused at time t1, every copy is stale from t1 + stale_fudge on: the slot is reused
  // only after that (slot_free_since_); a record of the old ID that is not stale yet restarts the
  // clock (Rec), since it may be stored again.
  uint16_t Id(uint32_t host, const std::string &id) {
    auto &m = ids_[host];
    auto it = m.find(id);
    if (it != m.end()) return it->second;
    uint16_t s;
    if (id_names_[host].size() < p_.n_services) {
      s = (uint16_t)id_names_[host].size();
      id_names_[host].push_back(id);
    } else {
      uint64_t used = 0;
      check(gx_owner_slots_in_use(e_, host, &used), "gx_owner_slots_in_use");
      auto &since = slot_free_since_[host];
      since.resize(p_.n_services, -1);
      const int64_t now = Now();
      s = p_.n_services;
      for (uint16_t k = 0; k < p_.n_services; k++) {
        if ((used >> k) & 1u) {
          since[k] = -1;
        } else {
          if (since[k] < 0) since[k] = now;  // first seen unused
          if (s == p_.n_services && now - since[k] > p_.stale_fudge_ns + 1000) s = k;
        }
      }
      if (s == p_.n_services) throw std::runtime_error("service table full: " + id);
      since[s] = -1;
      m.erase(id_names_[host][s]);  // the slot's old ID is forgotten, with its metadata
      id_names_[host][s] = id;
      const uint64_t key = (uint64_t)host * p_.n_services + s;
      if (names_.erase(key)) names_dirty_ = true;
      if (last_.erase(key)) codec_dirty_ = true;
      auto st = static_.find(host);
      if (st != static_.end() && st->second[s] != (uint16_t)GX_STATIC_BYTES_DEFAULT) {
        st->second[s] = (uint16_t)GX_STATIC_BYTES_DEFAULT;
        check(gx_set_static_bytes(e_, host, host + 1, st->second.data()), "gx_set_static_bytes");
      }
    }
    m[id] = s;
    return s;
  }
  gx_service Rec(const Service &svc) {
    uint32_t h = Host(svc.Hostname);
    if (!svc.Name.empty()) {  // remember the Name of the (host, ID) record for ByService
      std::string &n = names_[(uint64_t)h * p_.n_services + Id(h, svc.ID)];
      if (n != svc.Name) {
        n = svc.Name;
        names_dirty_ = true;
      }
    }
    gx_service r{};
    r.updated_ns = svc.Updated;
    r.host = h;
    r.svc = Id(h, svc.ID);
    {
      const uint64_t key = (uint64_t)h * p_.n_services + r.svc;
      auto it = last_.find(key);
      if (it == last_.end() || !SameMeta(it->second, svc)) codec_dirty_ = true;
      last_[key] = svc;
    }
    auto &since = slot_free_since_[h];
    if (r.svc < since.size() && since[r.svc] >= 0 &&
        svc.Updated >= Now() - p_.tombstone_lifespan_ns - p_.stale_fudge_ns)  // not IsStale: may be stored
      since[r.svc] = -1;
    r.status = (uint8_t)svc.Status;
    return r;
  }
  Service Svc(const gx_service &r) const {
    Service s;
    s.Hostname = r.host < host_names_.size() ? host_names_[r.host] : "host-" + std::to_string(r.host);
    s.ID = (r.host < id_names_.size() && r.svc < id_names_[r.host].size()) ? id_names_[r.host][r.svc]
                                                                             : "svc-" + std::to_string(r.svc);
    s.Updated = r.updated_ns;
    s.Status = r.status;
    auto it = names_.find((uint64_t)r.host * p_.n_services + r.svc);
    if (it != names_.end()) s.Name = it->second;
    auto lt = last_.find((uint64_t)r.host * p_.n_services + r.svc);
    if (lt != last_.end() && lt->second.ID == s.ID) {  // the metadata last seen for the record
      s.Image = lt->second.Image;
      s.Created = lt->second.Created;
      s.Ports = lt->second.Ports;
      s.ProxyMode = lt->second.ProxyMode;
      if (s.Name.empty()) s.Name = lt->second.Name;
    }
    return s;
  }
  static bool SameMeta(const Service &a, const Service &b) {
    bool ports = a.Ports.size() == b.Ports.size();
    for (size_t i = 0; ports && i < a.Ports.size(); i++)
      ports = a.Ports[i].Type == b.Ports[i].Type && a.Ports[i].Port == b.Ports[i].Port &&
              a.Ports[i].ServicePort == b.Ports[i].ServicePort && a.Ports[i].IP == b.Ports[i].IP;
    return ports && a.ID == b.ID && a.Hostname == b.Hostname && a.Name == b.Name && a.Image == b.Image &&
           a.Created == b.Created && a.ProxyMode == b.ProxyMode;
  }
  // Hands the engine the full-state codec's names (gx_set_names) when a record's metadata changed:
  // every host's name and every record's ID and JSON fragments (records never seen get placeholder
  // names the reference could not produce, so a peer's document never matches them).
  void SyncCodec(const std::string &cluster = "default") {
    if (!codec_dirty_ && cluster == codec_cluster_) return;
    const uint32_t H = p_.n_hosts, S = p_.n_services;
    std::string hosts, ids, pre, post;
    std::vector<uint64_t> ho(H + 1, 0), io((size_t)H * S + 1, 0), po((size_t)H * S + 1, 0), qo((size_t)H * S + 1, 0);
    for (uint32_t h = 0; h < H; h++) {
      hosts += h < host_names_.size() ? host_names_[h] : "\x01unused-host-" + std::to_string(h);
      ho[h + 1] = hosts.size();
      for (uint32_t j = 0; j < S; j++) {
        const uint64_t k = (uint64_t)h * S + j;
        Service svc;
        auto it = last_.find(k);
        if (it != last_.end()) svc = it->second;
        else svc.ID = "\x01unused-" + std::to_string(k), svc.Hostname = h < host_names_.size() ? host_names_[h] : "";
        const auto fr = json::fragments(svc);
        ids += svc.ID;
        pre += fr.first;
        post += fr.second;
        io[k + 1] = ids.size();
        po[k + 1] = pre.size();
        qo[k + 1] = post.size();
      }
    }
    gx_names n{};
    n.cluster_name = cluster.data();
    n.cluster_name_len = cluster.size();
    n.hosts = hosts.data();
    n.host_off = ho.data();
    n.ids = ids.data();
    n.id_off = io.data();
    n.pre = pre.data();
    n.pre_off = po.data();
    n.post = post.data();
    n.post_off = qo.data();
    check(gx_set_names(e_, &n), "gx_set_names");
    codec_dirty_ = false;
    codec_cluster_ = cluster;
  }
  // Decoding does not depend on the cluster name: keep the one the codec holds (an Encode with a
  // non-default name followed by a Decode would otherwise rebuild all H*S fragments twice).
  void SyncCodecForDecode() { SyncCodec(codec_cluster_.empty() ? std::string("default") : codec_cluster_); }
  // Hands the engine the Service.Name of every record (gx_set_service_names) when one changed.
  void SyncNames() {
    if (!names_dirty_) return;
    const uint64_t R = (uint64_t)p_.n_hosts * p_.n_services;
    std::string blob;
    std::vector<uint64_t> off(R + 1, 0);
    for (uint64_t r = 0; r < R; r++) {
      auto it = names_.find(r);
      if (it != names_.end()) blob += it->second;
      off[r + 1] = blob.size();
    }
    check(gx_set_service_names(e_, blob.data(), off.data()), "gx_set_service_names");
    names_dirty_ = false;
  }
  const std::vector<std::string> &HostNames() const { return host_names_; }
  // Encoded length of every field of svc's Service except Updated and Status (the Go side gets it
  // from len(svc.Encode()) minus those two); used by the byte-limited GetBroadcasts.
  void SetStaticBytes(const std::string &hostname, const std::string &id, uint16_t bytes) {
    uint32_t h = Host(hostname);
    uint16_t j = Id(h, id);
    std::vector<uint16_t> row(p_.n_services, (uint16_t)GX_STATIC_BYTES_DEFAULT);
    auto it = static_.find(h);
    if (it != static_.end()) row = it->second;
    row[j] = bytes;
    static_[h] = row;
    check(gx_set_static_bytes(e_, h, h + 1, row.data()), "gx_set_static_bytes");
  }
  std::vector<Service> Svcs(const std::vector<gx_service> &rs) const {
    std::vector<Service> out;
    for (auto &r : rs) out.push_back(Svc(r));
    return out;
  }

 private:
  gx_params p_;
  gx_engine *e_ = nullptr;
  std::map<std::string, uint32_t> hosts_;
  std::vector<std::string> host_names_;
  std::vector<std::map<std::string, uint16_t>> ids_;
  std::vector<std::vector<std::string>> id_names_;
  std::vector<std::vector<int64_t>> slot_free_since_;  // per owner slot: first time seen unused, -1
  std::map<uint32_t, std::vector<uint16_t>> static_;
  std::map<uint64_t, std::string> names_;  // record key -> Service.Name
  bool names_dirty_ = false;
  std::map<uint64_t, Service> last_;       // record key -> the last full Service seen (codec metadata)
  bool codec_dirty_ = true;
  std::string codec_cluster_;
};

namespace catalog {

// catalog.ServicesState of host `Hostname` (catalog/services_state.go:70-80).
class ServicesState {
 public:
  ServicesState(Cluster &c, const std::string &hostname) : c_(c), Hostname(hostname), self_(c.Host(hostname)) {}

  // AddServiceEntry (services_state.go:293-347)
  void AddServiceEntry(const Service &svc) {
    gx_service r = c_.Rec(svc);
    uint32_t v = self_;
    check(gx_add_service_entries(c_.engine(), &v, &r, 1, nullptr), "AddServiceEntry");
  }
  // Merge (services_state.go:367-373): another view of the same cluster
  void Merge(const ServicesState &other) { check(gx_merge(c_.engine(), self_, other.self_), "Merge"); }
  // Merge(otherState) with a state decoded from another node (catalog::Decode): AddServiceEntry of
  // each of its services in key order (services_state.go:367-373)
  void Merge(const std::vector<Service> &otherState) {
    std::vector<gx_service> rs;
    for (auto &svc : otherState) rs.push_back(c_.Rec(svc));
    if (!rs.empty())
      check(gx_merge_remote_state(c_.engine(), self_, rs.data(), (uint32_t)rs.size()), "Merge");
  }
  // UpdateService (services_state.go:137-140): the update reaches AddServiceEntry through the
  // ServiceMsgs loop (:129-135); here it is applied at once
  void UpdateService(const Service &svc) { AddServiceEntry(svc); }
  // Encode (services_state.go:115-125): the view's ServicesState JSON, the reference's bytes
  std::string Encode(const std::string &clusterName = "default") {
    c_.SyncCodec(clusterName);
    uint64_t n = 0;
    check(gx_local_state_json(c_.engine(), self_, nullptr, 0, &n), "Encode");
    std::string out(n, '\0');
    check(gx_local_state_json(c_.engine(), self_, n ? &out[0] : nullptr, n, &n), "Encode");
    return out;
  }
  // ExpireServer (services_state.go:150-192)
  void ExpireServer(const std::string &hostname) {
    check(gx_expire_server(c_.engine(), self_, c_.Host(hostname), nullptr), "ExpireServer");
  }
  // TombstoneOthersServices (services_state.go:635-683)
  std::vector<Service> TombstoneOthersServices() {
    std::vector<gx_service> out(4096);
    uint32_t n = 0;
    check(gx_tombstone_others(c_.engine(), self_, out.data(), (uint32_t)out.size(), &n), "TombstoneOthersServices");
    out.resize(n < out.size() ? n : out.size());
    return c_.Svcs(out);
  }
  // TombstoneServices(hostname, containerList) (services_state.go:685-715), hostname == self
  std::vector<Service> TombstoneServices(const std::vector<Service> &containerList) {
    std::vector<uint16_t> running;
    for (auto &s : containerList) running.push_back(c_.Id(self_, s.ID));
    std::vector<gx_service> out(256);
    uint32_t n = 0;
    check(gx_tombstone_services(c_.engine(), self_, running.data(), (uint32_t)running.size(), out.data(),
                                (uint32_t)out.size(), &n),
          "TombstoneServices");
    out.resize(n < out.size() ? n : out.size());
    return c_.Svcs(out);
  }
  // SendServices(services, looper(runCount)) (services_state.go:579-604)
  void SendServices(const std::vector<Service> &services, int runCount) {
    std::vector<gx_service> rs;
    for (auto &s : services) rs.push_back(c_.Rec(s));
    check(gx_send_services(c_.engine(), self_, rs.data(), (uint32_t)rs.size(), (uint32_t)runCount), "SendServices");
  }
  // One BroadcastServices looper body with fn (services_state.go:525-574)
  void BroadcastServices(const std::function<std::vector<Service>()> &fn) {
    std::vector<gx_service> rs;
    for (auto &s : fn()) rs.push_back(c_.Rec(s));
    check(gx_broadcast_services(c_.engine(), self_, rs.data(), (uint32_t)rs.size()), "BroadcastServices");
  }
  // One BroadcastTombstones looper body with fn (services_state.go:606-633)
  void BroadcastTombstones(const std::function<std::vector<Service>()> &fn) {
    std::vector<gx_service> rs;
    for (auto &s : fn()) rs.push_back(c_.Rec(s));
    check(gx_broadcast_tombstones(c_.engine(), self_, rs.data(), (uint32_t)rs.size()), "BroadcastTombstones");
  }
  // IsNewService (services_state.go:509-521)
  bool IsNewService(const Service &svc) {
    gx_service r = c_.Rec(svc);
    int x = 0;
    check(gx_is_new_service(c_.engine(), self_, &r, &x), "IsNewService");
    return x != 0;
  }
  // state.LastChanged
  int64_t LastChanged() const {
    int64_t t = 0;
    check(gx_read_last_changed(c_.engine(), self_, self_ + 1, &t), "LastChanged");
    return t;
  }
  // state.Servers[hostname].LastUpdated / LastChanged
  ServerTimes Times(const std::string &hostname) {
    gx_server_times t{};
    uint32_t o = c_.Host(hostname);
    check(gx_read_server_times(c_.engine(), self_, o, o + 1, &t), "ServerTimes");
    return {t.last_updated_ns, t.last_changed_ns};
  }
  // AddListener (:253-268): false when refused (an unbuffered channel, capacity 0)
  bool AddListener(const std::string &name, uint32_t capacity) {
    return gx_add_listener(c_.engine(), self_, ListenerId(name), capacity) == GX_OK;
  }
  // RemoveListener (:272-284): false = "no listener found with the name"
  bool RemoveListener(const std::string &name) {
    return gx_remove_listener(c_.engine(), self_, ListenerId(name)) == GX_OK;
  }
  // Receive everything buffered on a listener's channel, oldest first.
  std::vector<ChangeEvent> Receive(const std::string &name) {
    std::vector<gx_change_event> buf(GX_LISTENER_MAX_CAPACITY < 4096 ? GX_LISTENER_MAX_CAPACITY : 4096);
    std::vector<ChangeEvent> out;
    for (;;) {
      uint32_t n = 0;
      check(gx_listener_drain(c_.engine(), self_, ListenerId(name), buf.data(), (uint32_t)buf.size(), &n),
            "listener_drain");
      for (uint32_t i = 0; i < n; i++) out.push_back({c_.Svc(buf[i].service), (int)buf[i].previous_status, buf[i].time_ns});
      if (n < buf.size()) return out;
    }
  }
  // EachServiceSorted (catalog/view.go:14-26): by Updated; ties in key order (Go's sort.Sort
  // leaves them unspecified). Sorted by the engine (gx_each_service_sorted).
  std::vector<Service> EachServiceSorted() { return Sorted(GX_ALL_OWNERS); }
  // Server.SortedServices (view.go:48-58): one server's services by Updated.
  std::vector<Service> SortedServices(const std::string &hostname) { return Sorted(c_.Host(hostname)); }
  // SortedServers (view.go:82-92): the names of the servers this view holds, sorted.
  std::vector<std::string> SortedServers() {
    std::vector<std::string> out;
    for (auto &s : EachService())
      if (std::find(out.begin(), out.end(), s.Hostname) == out.end()) out.push_back(s.Hostname);
    std::sort(out.begin(), out.end());
    return out;
  }
  // ByService (services_state.go:738-748): services grouped by Service.Name, each group in
  // EachServiceSorted order (gx_by_service).
  std::map<std::string, std::vector<Service>> ByService() {
    c_.SyncNames();
    uint32_t n = 0;
    check(gx_by_service(c_.engine(), self_, nullptr, nullptr, 0, &n), "ByService");
    std::vector<gx_service> out(n ? n : 1);
    check(gx_by_service(c_.engine(), self_, out.data(), nullptr, n, &n), "ByService");
    std::map<std::string, std::vector<Service>> m;
    for (uint32_t i = 0; i < n; i++) {
      Service s = c_.Svc(out[i]);
      m[s.Name].push_back(s);
    }
    return m;
  }
  std::vector<Service> Sorted(uint32_t owner) {
    uint32_t n = 0;
    check(gx_each_service_sorted(c_.engine(), self_, owner, nullptr, 0, &n), "EachServiceSorted");
    std::vector<gx_service> out(n ? n : 1);
    check(gx_each_service_sorted(c_.engine(), self_, owner, out.data(), n, &n), "EachServiceSorted");
    out.resize(n);
    return c_.Svcs(out);
  }
  // state.Servers[hostname].Services[id], or nothing
  std::optional<Service> Get(const std::string &hostname, const std::string &id) {
    for (auto &s : EachService())
      if (s.Hostname == hostname && s.ID == id) return s;
    return std::nullopt;
  }
  bool HasServer(const std::string &hostname) {
    for (auto &s : EachService())
      if (s.Hostname == hostname) return true;
    return false;
  }
  // EachService (services_state.go:726-734), key order
  std::vector<Service> EachService() {
    uint32_t n = 0;
    check(gx_local_state(c_.engine(), self_, nullptr, 0, &n), "LocalState");
    std::vector<gx_service> out(n ? n : 1);
    check(gx_local_state(c_.engine(), self_, out.data(), n, &n), "LocalState");
    out.resize(n);
    return c_.Svcs(out);
  }
  // test hook: svc.Updated = ...; svc.Status = ... on the stored record (no merge rule)
  void Set(const Service &svc) {
    gx_service r = c_.Rec(svc);
    check(gx_write_slot(c_.engine(), self_, &r), "write_slot");
  }
  uint32_t index() const { return self_; }
  uint32_t ListenerId(const std::string &name) {
    auto it = listener_ids_.find(name);
    if (it != listener_ids_.end()) return it->second;
    uint32_t id = (uint32_t)listener_ids_.size();
    listener_ids_[name] = id;
    return id;
  }

 private:
  Cluster &c_;
  std::map<std::string, uint32_t> listener_ids_;

 public:
  const std::string Hostname;

 private:
  uint32_t self_;
};

// catalog.Decode (services_state.go:774-782): the services of a ServicesState JSON, document order.
// ok = false where the reference's UnmarshalJSON fails ("Decode() returns an error when handed
// junk", services_state_test.go:109-114); the services are then empty.
inline std::vector<Service> Decode(Cluster &c, const std::string &data, bool *ok = nullptr) {
  c.SyncCodecForDecode();
  std::vector<gx_service> out(64);
  uint32_t n = 0;
  gx_decode_stats ds{};
  int rc = gx_decode_state_json(c.engine(), data.data(), data.size(), out.data(), (uint32_t)out.size(), &n, &ds);
  if (rc == GX_OK && n > out.size()) {
    out.resize(n);
    rc = gx_decode_state_json(c.engine(), data.data(), data.size(), out.data(), n, &n, &ds);
  }
  if (ok) *ok = rc == GX_OK;
  if (rc != GX_OK) return {};
  out.resize(n);
  return c.Svcs(out);
}

}  // namespace catalog

// servicesDelegate (services_delegate.go:20-27) of one host.
class ServicesDelegate {
 public:
  ServicesDelegate(Cluster &c, catalog::ServicesState &state) : c_(c), state_(state) {}
  // NotifyMsg: one decoded packet's records (services_delegate.go:72-83, decode loop :46-56)
  void NotifyMsg(const std::vector<Service> &msg) {
    std::vector<gx_service> rs;
    for (auto &s : msg) rs.push_back(c_.Rec(s));
    check(gx_notify_msg(c_.engine(), state_.index(), rs.data(), (uint32_t)rs.size()), "NotifyMsg");
  }
  // GetBroadcasts with a record budget (services_delegate.go:85-144; packPacket :186-223). An
  // empty result is the reference's nil.
  std::vector<Service> GetBroadcasts(uint32_t limit_records = GX_LIMIT_DEFAULT) {
    std::vector<gx_service> out(256);
    uint32_t n = 0;
    check(gx_get_broadcasts(c_.engine(), state_.index(), limit_records, out.data(), (uint32_t)out.size(), &n),
          "GetBroadcasts");
    out.resize(n);
    return c_.Svcs(out);
  }
  // GetBroadcasts(overhead, limit) with the reference's byte limit (services_delegate.go:85-144,
  // packPacket :186-223); nil is an empty result.
  std::vector<Service> GetBroadcasts(int overhead, int limit) {
    const gx_params &p = c_.params();
    std::vector<gx_service> out(p.packet_cap + 2 * p.pending_cap);
    uint32_t n = 0;
    check(gx_get_broadcasts_bytes(c_.engine(), state_.index(), (uint32_t)overhead, (uint32_t)limit, out.data(),
                                  (uint32_t)out.size(), &n),
          "GetBroadcasts");
    out.resize(n);
    return c_.Svcs(out);
  }
  // LocalState (:146-151)
  std::vector<Service> LocalState(bool /*join*/) { return state_.EachService(); }
  // MergeRemoteState (:153-167)
  void MergeRemoteState(const std::vector<Service> &remote, bool /*join*/) {
    std::vector<gx_service> rs;
    for (auto &s : remote) rs.push_back(c_.Rec(s));
    check(gx_merge_remote_state(c_.engine(), state_.index(), rs.data(), (uint32_t)rs.size()), "MergeRemoteState");
  }
  // NotifyLeave (:173-176)
  void NotifyLeave(const std::string &node) {
    check(gx_notify_leave(c_.engine(), state_.index(), c_.Host(node)), "NotifyLeave");
  }

 private:
  Cluster &c_;
  catalog::ServicesState &state_;
};

}  // namespace sidecar
