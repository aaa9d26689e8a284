// The library's environment switches (A/B knobs of the kernel variants and a
// few diagnostics) as ONE process snapshot: every GG_* variable is copied when
// the snapshot is taken -- at the first lookup, at every gg_kron_create /
// gg_cg_create (a handle's configuration is latched when it is made) and by
// gg_knobs_reload -- so no launch path calls getenv.  Snapshots are never
// freed (a pointer knob() returned stays valid after a reload), and a reload
// that finds an environment it has seen before reuses that snapshot, so a
// loop creating handles does not grow memory: one snapshot per distinct
// GG_* environment.
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gg_internal.h"

extern char** environ;

namespace gg {

namespace {
typedef std::map<std::string, std::string> Snapshot;
std::mutex g_mu;
std::vector<std::unique_ptr<Snapshot>> g_all;   // every distinct snapshot (kept alive)
const Snapshot* g_cur = nullptr;

const Snapshot* take() {
  std::unique_ptr<Snapshot> s(new Snapshot());
  for (char** e = environ; e && *e; ++e) {
    if (strncmp(*e, "GG_", 3) != 0) continue;
    const char* eq = strchr(*e, '=');
    if (eq) (*s)[std::string(*e, eq - *e)] = std::string(eq + 1);
  }
  for (const auto& old : g_all)
    if (*old == *s) return old.get();
  g_all.push_back(std::move(s));
  return g_all.back().get();
}
}  // namespace

void knobs_reload() {
  std::lock_guard<std::mutex> lk(g_mu);
  g_cur = take();
}

const char* knob(const char* name) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_cur == nullptr) g_cur = take();
  auto it = g_cur->find(name);
  return it == g_cur->end() ? nullptr : it->second.c_str();
}

}  // namespace gg

extern "C" int gg_knobs_reload(void) {
  return gg::guard([&] { gg::knobs_reload(); });
}
