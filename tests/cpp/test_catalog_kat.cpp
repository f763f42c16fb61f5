// Reference KATs restated in C++ against the host mirror (include/sidecar/catalog.hpp), i.e. the
// same method names as catalog/services_state_test.go and services_delegate_test.go. Linked
// against either gx.h implementation (CPU oracle for the CPU suite, libgx.so on the GPU).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "sidecar/catalog.hpp"

using sidecar::Cluster;
using sidecar::Service;
using sidecar::ServicesDelegate;
using sidecar::catalog::ServicesState;

static int failures = 0, checks = 0;
#define So(cond)                                                                  \
  do {                                                                            \
    checks++;                                                                     \
    if (!(cond)) {                                                                \
      failures++;                                                                 \
      std::fprintf(stderr, "%s:%d: %s: FAILED %s\n", __FILE__, __LINE__, cur, #cond); \
    }                                                                             \
  } while (0)
static const char *cur = "";

static const int64_t SEC = 1000000000ll, MIN = 60 * SEC, HOUR = 60 * MIN;
static const std::string hostname = "shakespeare", anotherHostname = "chaucer", local = "localhost";

static gx_params params() {
  gx_params p = Cluster::Defaults(8, 8);
  p.t0_ns = 1700000000ll * SEC;
  p.retransmit_rounds = 0;  // state.tombstoneRetransmit = 1ns
  p.queue_cap = 64;
  return p;
}

// Test_ServicesStateWithData (services_state_test.go:82-321)
static void test_services_state_with_data() {
  {
    cur = "Merges in a new service (:126-133)";
    Cluster c(params());
    ServicesState state(c, local);
    Service svc{"deadbeef123", anotherHostname, c.Now(), sidecar::ALIVE};
    So(!state.HasServer(anotherHostname));
    state.AddServiceEntry(svc);
    So(state.HasServer(anotherHostname));
    So(state.Get(anotherHostname, svc.ID).has_value());
  }
  {
    cur = "Doesn't merge an update that is older than what we have (:135-155)";
    Cluster c(params());
    ServicesState state(c, local);
    Service svc{"deadbeef123", anotherHostname, c.Now(), sidecar::ALIVE};
    state.AddServiceEntry(svc);
    Service stale = svc;
    stale.Updated = svc.Updated - MIN;
    state.AddServiceEntry(stale);
    So(state.Get(anotherHostname, svc.ID)->Updated == svc.Updated);
  }
  {
    cur = "Doesn't merge an update that is past the tombstone lifespan (:157-175)";
    Cluster c(params());
    ServicesState state(c, local);
    int64_t base = c.Now();
    c.Advance(1);  // the reference re-reads time.Now() inside IsStale
    Service stale{"deadbeef123", anotherHostname, base - MIN - 3 * HOUR, sidecar::ALIVE};
    state.AddServiceEntry(stale);
    So(!state.HasServer(anotherHostname));
  }
  {
    cur = "Retransmits a packet when the state changes (:214-225)";
    Cluster c(params());
    ServicesState state(c, local);
    ServicesDelegate delegate(c, state);
    Service svc{"deadbeef123", anotherHostname, c.Now(), sidecar::ALIVE};
    state.AddServiceEntry(svc);
    So(delegate.GetBroadcasts().size() == 1);  // catch the retransmit from the initial add
    c.Advance(1);
    svc.Status = sidecar::TOMBSTONE;  // svc.Tombstone()
    svc.Updated = c.Now();
    state.AddServiceEntry(svc);
    auto packet = delegate.GetBroadcasts();
    So(packet.size() == 1 && packet[0] == svc);
  }
  {
    cur = "Doesn't retransmit an add of a new service for this host (:227-243)";
    Cluster c(params());
    ServicesState state(c, hostname);
    ServicesDelegate delegate(c, state);
    state.AddServiceEntry(Service{"deadbeef123", hostname, c.Now(), sidecar::ALIVE});
    So(delegate.GetBroadcasts().empty());
  }
  {
    cur = "Sets a service's status to DRAINING (:245-256)";
    Cluster c(params());
    ServicesState state(c, local);
    Service svc{"deadbeef123", anotherHostname, c.Now(), sidecar::ALIVE};
    state.AddServiceEntry(svc);
    c.Advance(1);
    svc.Status = sidecar::DRAINING;
    svc.Updated = c.Now();
    state.AddServiceEntry(svc);
    So(state.Get(anotherHostname, svc.ID)->Status == sidecar::DRAINING);
  }
  {
    cur = "Doesn't mark a DRAINING service as ALIVE (:258-270)";
    Cluster c(params());
    ServicesState state(c, local);
    Service svc{"deadbeef123", anotherHostname, c.Now(), sidecar::DRAINING};
    state.AddServiceEntry(svc);
    c.Advance(1);
    svc.Status = sidecar::ALIVE;
    svc.Updated = c.Now();
    state.AddServiceEntry(svc);
    So(state.Get(anotherHostname, svc.ID)->Status == sidecar::DRAINING);
  }
  {
    cur = "Merge() merges state we care about from other state structs (:299-308)";
    Cluster c(params());
    ServicesState firstState(c, "first"), secondState(c, "second");
    firstState.AddServiceEntry(Service{"deadbeef123", anotherHostname, c.Now(), sidecar::ALIVE});
    secondState.Merge(firstState);
    So(secondState.EachService() == firstState.EachService());
  }
}

// Test_TrackingAndBroadcasting (services_state_test.go:323-570)
static void test_tracking_and_broadcasting() {
  gx_params p = params();
  {
    cur = "The correct number of messages are sent (:345-353)";
    Cluster c(p);
    ServicesState state(c, hostname);
    ServicesDelegate d(c, state);
    std::vector<Service> services{{"deadbeef123", hostname, c.Now(), sidecar::ALIVE},
                                  {"deadbeef101", hostname, c.Now(), sidecar::ALIVE}};
    state.SendServices(services, 5);
    int n = 0;
    while (!d.GetBroadcasts().empty()) n++;
    So(n == 5);
  }
  {
    cur = "New services are serialized into the channel (:368-378)";
    Cluster c(p);
    ServicesState state(c, hostname);
    ServicesDelegate d(c, state);
    std::vector<Service> services{{"deadbeef123", hostname, c.Now(), sidecar::ALIVE},
                                  {"deadbeef101", hostname, c.Now(), sidecar::ALIVE}};
    state.BroadcastServices([&] { return services; });
    So(d.GetBroadcasts() == services);
  }
  {
    cur = "Puts a nil into the broadcasts channel when no services (:380-386)";
    Cluster c(p);
    ServicesState state(c, hostname);
    ServicesDelegate d(c, state);
    state.BroadcastServices([] { return std::vector<Service>{}; });
    So(d.GetBroadcasts().empty());
  }
  {
    cur = "All of the tombstones are serialized into the channel (:388-400)";
    Cluster c(p);
    ServicesState state(c, hostname);
    ServicesDelegate d(c, state);
    Service junk{"runs", hostname, c.Now(), sidecar::ALIVE};
    std::vector<Service> services{{"deadbeef123", hostname, c.Now(), sidecar::ALIVE},
                                  {"deadbeef101", hostname, c.Now(), sidecar::ALIVE}};
    state.AddServiceEntry(junk);
    for (auto &s : services) state.AddServiceEntry(s);
    state.BroadcastTombstones([&] { return services; });
    auto b = d.GetBroadcasts();
    So(b.size() == 2);
    for (auto &x : b) So(x.ID == "runs" && x.Status == sidecar::TOMBSTONE);
  }
  {
    cur = "The timestamp is incremented on each subsequent service broadcast background run (:402-424)";
    Cluster c(p);
    ServicesState state(c, hostname);
    ServicesDelegate d(c, state);
    Service s1{"deadbeef123", hostname, c.Now(), sidecar::TOMBSTONE};
    state.SendServices({s1}, 2);
    So(d.GetBroadcasts()[0].Updated == s1.Updated);
    So(d.GetBroadcasts()[0].Updated == s1.Updated + 50);
  }
  {
    cur = "Alive services have a lifespan and then are tombstoned (:480-492)";
    Cluster c(p);
    ServicesState state(c, hostname);
    Service s1{"deadbeef123", hostname, c.Now(), sidecar::ALIVE};
    state.AddServiceEntry(s1);
    int64_t stamp = s1.Updated - 80 * SEC - 5 * SEC;
    state.Set(Service{s1.ID, hostname, stamp, sidecar::ALIVE});
    state.TombstoneOthersServices();
    auto got = state.Get(hostname, s1.ID);
    So(got->Status == sidecar::TOMBSTONE && got->Updated == stamp + SEC);
  }
  {
    cur = "Draining services are not tombstoned before their lifespan expires (:509-522)";
    Cluster c(p);
    ServicesState state(c, hostname);
    Service s1{"deadbeef123", hostname, c.Now(), sidecar::DRAINING};
    state.AddServiceEntry(s1);
    int64_t stamp = s1.Updated - 80 * SEC - 5 * SEC;
    state.Set(Service{s1.ID, hostname, stamp, sidecar::DRAINING});
    state.TombstoneOthersServices();
    So(state.Get(hostname, s1.ID)->Status == sidecar::DRAINING);
  }
  {
    cur = "Can detect new services or newly changed services (:552-559)";
    Cluster c(p);
    ServicesState state(c, hostname);
    state.AddServiceEntry(Service{"deadbeef123", hostname, c.Now(), sidecar::UNHEALTHY});
    So(state.IsNewService(Service{"deadbeef123", hostname, c.Now(), sidecar::ALIVE}));
    So(!state.IsNewService(Service{"deadbeef123", hostname, c.Now(), sidecar::TOMBSTONE}));
  }
}

// Test_ClusterMembershipManagement (services_state_test.go:675-731)
static void test_cluster_membership() {
  {
    cur = "ExpireServer() tombstones all services for a server (:691-714)";
    Cluster c(params());
    ServicesState state(c, hostname);
    ServicesDelegate d(c, state);
    state.AddServiceEntry(Service{"deadbeef123", hostname, c.Now(), sidecar::ALIVE});
    state.AddServiceEntry(Service{"deadbeef101", hostname, c.Now(), sidecar::ALIVE});
    state.ExpireServer(hostname);
    auto expired = d.GetBroadcasts();
    So(expired.size() == 2);
    for (auto &x : expired) So(x.Status == sidecar::TOMBSTONE);
  }
  {
    cur = "does not announce services for hosts with no alive services (:722-729)";
    Cluster c(params());
    ServicesState state(c, hostname);
    ServicesDelegate d(c, state);
    state.AddServiceEntry(Service{"deadbeef123", hostname, c.Now(), sidecar::TOMBSTONE});
    state.ExpireServer(hostname);
    So(state.EachService().size() == 1);
    So(d.GetBroadcasts().empty());
  }
}

// Test_GetBroadcasts (services_delegate_test.go:40-103)
static void test_get_broadcasts() {
  Cluster c(params());
  ServicesState state(c, local);
  ServicesDelegate delegate(c, state);
  cur = "Returns nil when there is nothing to send (:41-43)";
  So(delegate.GetBroadcasts(6).empty());
  cur = "Returns what's in the channel (:54-63)";
  std::vector<Service> bCast{{"d419fa7ad1a7", "docker2", 1425431566669648453ll, sidecar::ALIVE},
                             {"deadbeefabba", "docker2", 1425431566669648453ll, sidecar::ALIVE}};
  state.SendServices(bCast, 1);
  So(delegate.GetBroadcasts(6) == bCast);
  cur = "NotifyMsg merges the packet (:72-83)";
  c.Advance(1);
  delegate.NotifyMsg({Service{"feedface", "docker3", c.Now(), sidecar::ALIVE}});
  So(state.HasServer("docker3"));
  cur = "NotifyLeave expires the node (:173-176)";
  delegate.NotifyLeave("docker3");
  So(state.Get("docker3", "feedface")->Status == sidecar::TOMBSTONE);
}

// Test_GetBroadcasts "Many runs with leftovers" (services_delegate_test.go:88-103) with the
// reference's byte limits: the fixture messages are 225 / 225 / 214 bytes long.
static void test_get_broadcasts_bytes() {
  Cluster c(params());
  ServicesState state(c, local);
  ServicesDelegate delegate(c, state);
  const int64_t t46 = 1425431566669648453ll, t32 = 1425431552630357657ll;
  // 225 = static + len("\"2015-03-04T01:12:46.669648453Z\"") 32 + len("0") 1
  c.SetStaticBytes("docker2", "d419fa7ad1a7", 225 - 33);
  c.SetStaticBytes("docker2", "deadbeefabba", 225 - 33);
  c.SetStaticBytes("docker1", "1b3295bf300f", 214 - 33);
  std::vector<Service> bCast{{"d419fa7ad1a7", "docker2", t46, sidecar::ALIVE},
                             {"deadbeefabba", "docker2", t46, sidecar::ALIVE}};
  std::vector<Service> bCast2{{"1b3295bf300f", "docker1", t32, sidecar::ALIVE},
                              {"deadbeefabba", "docker2", t46, sidecar::ALIVE}};
  cur = "pendingBroadcasts = bCast (nothing fits in 3/100)";
  state.SendServices(bCast, 1);
  So(delegate.GetBroadcasts(3, 100).empty());
  cur = "channel <- bCast2 ++ bCast; 3/100 sends nothing";
  std::vector<Service> both = bCast2;
  both.insert(both.end(), bCast.begin(), bCast.end());
  state.SendServices(both, 1);
  So(delegate.GetBroadcasts(3, 100).empty());
  cur = "3/300: one message fits";
  auto one = delegate.GetBroadcasts(3, 300);
  So(one.size() == 1 && one[0] == bCast2[0]);
  So(delegate.GetBroadcasts(3, 100).empty());
  cur = "3/1398: the other five";
  auto five = delegate.GetBroadcasts(3, 1398);
  So(five.size() == 5 && five[0] == bCast2[1] && five[1] == bCast[0] && five[2] == bCast[1]);
  So(delegate.GetBroadcasts(3, 1398).empty());
}

// Server times, state.LastChanged and listeners (services_state_test.go:177-212, :572-626)
static void test_change_bookkeeping() {
  Cluster c(params());
  ServicesState state(c, local);
  const int64_t t0 = c.Now();
  Service svc{"deadbeef123", "chaucer", t0, sidecar::ALIVE};
  cur = "NewServer / NewServicesState start at Unix(0)";
  So(state.LastChanged() == 0 && state.Times("chaucer").LastUpdated == 0);
  cur = "AddListener refuses an unbuffered channel";
  So(!state.AddListener("bad", 0));
  So(state.AddListener("listener1", 1) && state.AddListener("listener2", 8));
  cur = "a new service moves LastChanged; the listeners hear it";
  state.AddServiceEntry(svc);
  So(state.LastChanged() == t0 && state.Times("chaucer").LastChanged == t0);
  cur = "a newer record with the same status moves only LastUpdated";
  svc.Updated = t0 + 5;
  state.AddServiceEntry(svc);
  So(state.Times("chaucer").LastUpdated == t0 + 5 && state.LastChanged() == t0);
  cur = "a status change moves LastChanged and is an event (previous status ALIVE)";
  svc.Updated = t0 + 9;
  svc.Status = sidecar::TOMBSTONE;
  state.AddServiceEntry(svc);
  So(state.LastChanged() == t0 + 9);
  auto e1 = state.Receive("listener1"), e2 = state.Receive("listener2");
  So(e1.size() == 1 && e1[0].PreviousStatus == sidecar::UNKNOWN);  // channel of 1: the second was dropped
  So(e2.size() == 2 && e2[1].PreviousStatus == sidecar::ALIVE && e2[1].Svc == svc && e2[1].Time == t0 + 9);
  cur = "RemoveListener reports a missing one";
  So(state.RemoveListener("listener1") && !state.RemoveListener("listener1"));
  cur = "EachServiceSorted orders by Updated";
  state.AddServiceEntry(Service{"older", "chaucer", t0 - 100, sidecar::ALIVE});
  auto sorted = state.EachServiceSorted();
  So(sorted.size() == 2 && sorted[0].ID == "older");
}

// Test_ServerSorting (catalog/view_test.go:17-95) and ByService (services_state.go:738-748)
static void test_view_sorting() {
  const std::string h1 = "shakespeare", h2 = "chaucer", h3 = "bocaccio";
  const std::string id1 = "deadbeef123", id2 = "deadbeef101", id3 = "deadbeef105";
  Cluster c(params());
  ServicesState state(c, local);
  const int64_t base = c.Now();
  state.AddServiceEntry(Service{id1, h1, base + 5 * SEC, sidecar::ALIVE, "web"});
  state.AddServiceEntry(Service{id2, h2, base, sidecar::ALIVE, "db"});
  state.AddServiceEntry(Service{id3, h3, base + 10 * SEC, sidecar::ALIVE, "web"});
  {
    cur = "Returns a list of Servers sorted by Name (view_test.go:36-48)";
    auto names = state.SortedServers();
    So(names.size() == 3 && names[0] == "bocaccio" && names[1] == "chaucer" && names[2] == "shakespeare");
  }
  {
    cur = "Returns a list of Services sorted by Updates (view_test.go:50-69)";
    ServicesState s2(c, "view2");
    s2.AddServiceEntry(Service{id3, h3, base + 10 * SEC, sidecar::ALIVE});
    s2.AddServiceEntry(Service{id2, h3, base, sidecar::ALIVE});
    s2.AddServiceEntry(Service{id1, h3, base + 5 * SEC, sidecar::ALIVE});
    auto v = s2.SortedServices(h3);
    So(v.size() == 3 && v[0].ID == id2 && v[1].ID == id1 && v[2].ID == id3);
  }
  {
    cur = "Returs a list of Services sorted on sorted Servers (view_test.go:71-91)";
    state.AddServiceEntry(Service{id1, h3, base + 5 * SEC, sidecar::ALIVE, "web"});
    state.AddServiceEntry(Service{id2, h3, base, sidecar::ALIVE, "db"});
    state.AddServiceEntry(Service{id3, h3, base + 10 * SEC, sidecar::ALIVE, "web"});
    std::vector<std::string> ids;
    for (auto &s : state.EachServiceSorted()) ids.push_back(s.ID);
    const std::vector<std::string> should = {id2, id2, id1, id1, id3};
    So(ids == should);
  }
  {
    cur = "ByService groups by Service.Name in EachServiceSorted order (services_state.go:738-748)";
    auto m = state.ByService();
    So(m.size() == 2 && m.count("db") && m.count("web"));
    So(m["db"].size() == 2 && m["db"][0].Updated == base && m["db"][1].Updated == base);
    So(m["web"].size() == 3 && m["web"][0].ID == id1 && m["web"][2].ID == id3);
  }
  {
    cur = "A server and services first seen by gossip are created (services_state.go:310-318)";
    ServicesState s3(c, "newcomer-view");
    ServicesDelegate del(c, s3);
    del.NotifyMsg({Service{"fresh-1", "brand-new-host", base, sidecar::ALIVE}, Service{"fresh-2", "brand-new-host", base + SEC, sidecar::ALIVE}});
    So(s3.HasServer("brand-new-host"));
    So(s3.Get("brand-new-host", "fresh-2").has_value());
    auto v = s3.SortedServices("brand-new-host");
    So(v.size() == 2 && v[0].ID == "fresh-1");
  }
}

// Dynamic key space of the host mirror: a new ID takes a free slot, and once the owner's S slots
// are taken, one whose record every view has garbage-collected (services_state.go:645-653).
static void test_slot_reuse() {
  gx_params p = params();
  p.n_services = 2;
  Cluster c(p);
  ServicesState state(c, local);
  const std::string h = "bocaccio";
  const int64_t t = c.Now();
  state.AddServiceEntry(Service{"a1", h, t, sidecar::ALIVE});
  state.AddServiceEntry(Service{"a2", h, t, sidecar::ALIVE});
  {
    cur = "A full table of live services refuses a third ID";
    bool threw = false;
    try {
      state.AddServiceEntry(Service{"a3", h, t, sidecar::ALIVE});
    } catch (const std::runtime_error &) {
      threw = true;
    }
    So(threw);
  }
  auto refused = [&](const Service &svc) {
    try {
      state.AddServiceEntry(svc);
    } catch (const std::runtime_error &) {
      return true;
    }
    return false;
  };
  {
    cur = "A collected slot is not reused while a queued copy of its tombstone can still merge";
    state.AddServiceEntry(Service{"a1", h, t + SEC, sidecar::TOMBSTONE});
    state.AddServiceEntry(Service{"a2", h, t + SEC, sidecar::TOMBSTONE});
    // just past TOMBSTONE_LIFESPAN: collected (:645-653) but not yet stale (+1 min, service.go:68-71)
    c.Advance((3 * HOUR + 2 * SEC) / p.round_ns);
    state.TombstoneOthersServices();
    So(!state.Get(h, "a1").has_value() && !state.Get(h, "a2").has_value());
    So(refused(Service{"a3", h, c.Now(), sidecar::ALIVE}));
    // a peer still had a1's tombstone queued: it merges as a1, not as a new ID on a1's slot
    ServicesDelegate peer(c, state);
    peer.NotifyMsg({Service{"a1", h, t + SEC, sidecar::TOMBSTONE}});
    So(state.Get(h, "a1").has_value() && state.Get(h, "a1")->Status == sidecar::TOMBSTONE);
    So(!state.Get(h, "a3").has_value());
  }
  {
    cur = "After the tombstones are collected everywhere, a new ID reuses a slot";
    c.Advance(2 * MIN / p.round_ns);  // a2's slot: unused for longer than the stale fudge
    state.TombstoneOthersServices();  // collects a1's tombstone again (:645-653)
    So(!state.Get(h, "a1").has_value() && !state.Get(h, "a2").has_value());
    state.AddServiceEntry(Service{"a3", h, c.Now(), sidecar::ALIVE});
    So(state.Get(h, "a3").has_value());
    auto v = state.SortedServices(h);
    So(v.size() == 1 && v[0].ID == "a3");
    So(refused(Service{"a4", h, c.Now(), sidecar::ALIVE}));  // a1's slot: its clock restarted by the merge
    ServicesDelegate peer(c, state);
    peer.NotifyMsg({Service{"a1", h, t + SEC, sidecar::TOMBSTONE}});  // stale by now: dropped
    So(!state.Get(h, "a1").has_value());
    c.Advance(2 * MIN / p.round_ns);
    state.AddServiceEntry(Service{"a4", h, c.Now(), sidecar::ALIVE});
    So(state.Get(h, "a4").has_value() && state.SortedServices(h).size() == 2);
  }
}

// Encode / Decode / Merge(decoded state) / UpdateService (services_state_test.go:102-115, :299-308;
// services_state.go:115-140, 367-373, 774-782). The expected Service bytes are the Python codec's
// (sidecar_amd/codec.py service_json, pinned to the services_delegate_test.go:15-20 records).
static std::string full_json(const Service &s) {
  auto fr = sidecar::json::fragments(s);
  return fr.first + sidecar::json::time(s.Updated) + fr.second + std::to_string(s.Status) + "}";
}
static void test_codec() {
  {
    cur = "Service JSON: ffjson field order, HTML-escaped strings, RFC3339Nano";
    Service a{"deadbeef123", "chaucer", 1700000000000000000ll, sidecar::TOMBSTONE, "web<1>", "img:1",
              1425431552630357657ll, {{"tcp", 8080, 10001, "192.168.1.1"}, {"udp", 53, 0, ""}}, "http"};
    So(full_json(a) ==
       "{\"ID\":\"deadbeef123\",\"Name\":\"web\\u003c1\\u003e\",\"Image\":\"img:1\",\"Created\":"
       "\"2015-03-04T01:12:32.630357657Z\",\"Hostname\":\"chaucer\",\"Ports\":[{\"Type\":\"tcp\",\"Port\":8080,"
       "\"ServicePort\":10001,\"IP\":\"192.168.1.1\"},{\"Type\":\"udp\",\"Port\":53,\"ServicePort\":0,\"IP\":\"\"}],"
       "\"Updated\":\"2023-11-14T22:13:20Z\",\"ProxyMode\":\"http\",\"Status\":1}");
    Service b{"x\xe2\x80\xa8\xc3\xa9", "h", 1700000000123000000ll, sidecar::UNHEALTHY};
    So(full_json(b) ==
       "{\"ID\":\"x\\u2028\xc3\xa9\",\"Name\":\"\",\"Image\":\"\",\"Created\":\"1970-01-01T00:00:00Z\",\"Hostname\":"
       "\"h\",\"Ports\":null,\"Updated\":\"2023-11-14T22:13:20.123Z\",\"ProxyMode\":\"\",\"Status\":2}");
    Service c{"a\x01\"b\\", "h\xc3\xbf", 1, sidecar::ALIVE, "n"};
    c.Created = -1;
    So(full_json(c) ==
       "{\"ID\":\"a\\u0001\\\"b\\\\\",\"Name\":\"n\",\"Image\":\"\",\"Created\":\"1969-12-31T23:59:59.999999999Z\","
       "\"Hostname\":\"h\xc3\xbf\",\"Ports\":null,\"Updated\":\"1970-01-01T00:00:00.000000001Z\",\"ProxyMode\":\"\","
       "\"Status\":0}");
    So(sidecar::json::quote("\xff") == "\"\\ufffd\"");
  }
  {
    cur = "Encode() generates JSON that we can Decode() (:102-107)";
    Cluster c(params());
    ServicesState state(c, hostname);
    Service svc{"deadbeef123", hostname, c.Now(), sidecar::ALIVE, "web", "img"};
    state.AddServiceEntry(svc);
    std::string enc = state.Encode();
    So(enc.rfind("{\"Servers\":{\"shakespeare\":{\"Name\":\"shakespeare\",\"Services\":{\"deadbeef123\":", 0) == 0);
    So(enc.find(full_json(svc)) != std::string::npos);
    bool ok = false;
    auto decoded = sidecar::catalog::Decode(c, enc, &ok);
    So(ok && decoded.size() == 1 && decoded[0] == svc && decoded[0].Hostname == hostname);
    So(decoded.size() == 1 && decoded[0].Name == "web" && decoded[0].Image == "img");
  }
  {
    cur = "Decode() returns an error when handed junk (:109-114)";
    Cluster c(params());
    ServicesState state(c, hostname);
    state.AddServiceEntry(Service{"deadbeef123", hostname, c.Now(), sidecar::ALIVE});
    bool ok = true;
    auto decoded = sidecar::catalog::Decode(c, "asdf", &ok);
    So(!ok && decoded.empty());
  }
  {
    cur = "Merge() of a decoded remote state (:299-308 through Encode/Decode)";
    Cluster c(params());
    ServicesState firstState(c, "first"), secondState(c, "second");
    firstState.AddServiceEntry(Service{"deadbeef123", anotherHostname, c.Now(), sidecar::ALIVE});
    firstState.AddServiceEntry(Service{"cafe", hostname, c.Now(), sidecar::DRAINING});
    auto other = sidecar::catalog::Decode(c, firstState.Encode());
    So(other.size() == 2);
    secondState.Merge(other);
    So(secondState.EachService() == firstState.EachService());
  }
  {
    cur = "UpdateService() reaches AddServiceEntry (services_state.go:129-140)";
    Cluster c(params());
    ServicesState state(c, local);
    Service svc{"deadbeef123", anotherHostname, c.Now(), sidecar::ALIVE};
    state.UpdateService(svc);
    So(state.Get(anotherHostname, svc.ID).has_value());
    c.Advance(1);
    svc.Status = sidecar::TOMBSTONE;
    svc.Updated = c.Now();
    state.UpdateService(svc);
    So(state.Get(anotherHostname, svc.ID)->Status == sidecar::TOMBSTONE);
  }
}

int main() {
  test_slot_reuse();
  test_view_sorting();
  test_services_state_with_data();
  test_tracking_and_broadcasting();
  test_cluster_membership();
  test_get_broadcasts();
  test_get_broadcasts_bytes();
  test_change_bookkeeping();
  test_codec();
  std::printf("backend=%s checks=%d failures=%d\n", gx_backend(), checks, failures);
  return failures ? 1 : 0;
}
