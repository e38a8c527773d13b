// serve_bench.cpp -- measurement infrastructure (not the product): the
// drop-in read/6 serving path driven the way AntidoteDB drives it, from
// native threads through the C ABI only (include/antidote_gpu.h), so no
// interpreter sits between the callers and the library.
//
// `parts` partitions (materializer_vnodes) on one GPU, each with its own
// engine-owned counter_pn op log of `keys` keys x `ops` ops
// (agn_oplog_append, op ids from the per-key counter), its own cached batcher
// (agn_batcher_create_cached: read/6 = snapshot-cache lookup -> materialize
// from the cached base -> store_ss / GC, on the batcher's stream), `threads`
// read servers (READ_CONCURRENCY = 20, include/antidote.hrl:28) issuing reads
// of random keys at the partition's current clock, and optionally one writer
// (the vnode's update/2) appending `wps` updates per second.  `hot` > 0
// restricts reads and writes to keys [0, hot): repeated reads of growing keys,
// so snapshot-cache hits, stores and the GC run.  Reports reads/s over all
// partitions, per-read latency percentiles, mean batch size and read
// statuses as one JSON line.
//
// sparse=1 builds the logs the way the Erlang NIF does (nif_part_open,
// nif/antidote_gpu_nif.c): presence masks on every clock (the op rows, the
// reads' R, LastOpCt), `dcs` columns of which the first `present` are
// interned DCs (the rest absent from every dict clock).
//
// type=set|register serves set_aw / register_mv partitions instead (16
// elements / values per key; an add / assign removes / overrides the key's
// previous token of it, as the CRDTs' downstream does): their snapshot states
// live in the cache's device arena.
//
//   serve_bench [type=counter|set|register] [keys=N] [ops=N] [dcs=N] [present=N]
//               [sparse=0|1] [parts=N] [threads=N] [reads=N] [batch=N] [wait=US]
//               [wps=N] [hot=N] [crash=1]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <ucontext.h>
#include <unistd.h>

#include "antidote_gpu.h"

namespace {

// crash=1: a SIGSEGV / SIGBUS handler (installed after agn_open, so it
// replaces any a profiler's tool library installed) that names the faulting
// address, the PC's shared object + symbol (dladdr), a backtrace, and the
// /proc/self/maps lines around both -- where a crash under a profiler comes
// from.  Only async-signal-tolerant calls on the raw fd; then the default
// action (core) is restored and the signal re-raised.
void put(const char *s) { (void)!write(2, s, std::strlen(s)); }
void put_hex(const char *label, uint64_t v) {
    char b[64];
    std::snprintf(b, sizeof b, "%s0x%llx\n", label, (unsigned long long)v);
    put(b);
}
void maps_near(uint64_t a) {
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd < 0) return;
    static char buf[1 << 20];
    ssize_t n = 0, r;
    while (n < (ssize_t)sizeof buf - 1 && (r = read(fd, buf + n, sizeof buf - 1 - n)) > 0) n += r;
    close(fd);
    buf[n] = 0;
    char *line = buf;
    while (line && *line) {
        char *nl = std::strchr(line, '\n');
        if (nl) *nl = 0;
        unsigned long long lo = 0, hi = 0;
        if (std::sscanf(line, "%llx-%llx", &lo, &hi) == 2 && a + (2ull << 20) >= lo && a < hi + (2ull << 20)) {
            put("  maps: ");
            put(line);
            put("\n");
        }
        if (nl) *nl = '\n';
        line = nl ? nl + 1 : nullptr;
    }
}
void on_crash(int sig, siginfo_t *si, void *ctx) {
    const uint64_t addr = (uint64_t)si->si_addr;
    const uint64_t pc = (uint64_t)((ucontext_t *)ctx)->uc_mcontext.gregs[REG_RIP];
    put(sig == SIGSEGV ? "serve_bench: SIGSEGV\n" : "serve_bench: SIGBUS\n");
    put_hex("  fault address: ", addr);
    put_hex("  pc: ", pc);
    put_hex("  thread: ", (uint64_t)gettid());
    Dl_info di;
    if (dladdr((void *)pc, &di)) {
        put("  pc object: ");
        put(di.dli_fname ? di.dli_fname : "?");
        put("\n  pc symbol: ");
        put(di.dli_sname ? di.dli_sname : "?");
        put("\n");
        put_hex("  pc - object base: ", pc - (uint64_t)di.dli_fbase);
    }
    void *bt[64];
    const int nb = backtrace(bt, 64);
    put("  backtrace:\n");
    backtrace_symbols_fd(bt, nb, 2);
    put("  mappings near the fault address:\n");
    maps_near(addr);
    put("  mappings near the pc:\n");
    maps_near(pc);
    signal(sig, SIG_DFL);
    raise(sig);
}
void install_crash_handler() {
    struct sigaction sa;
    std::memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_crash;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigaction(SIGSEGV, &sa, nullptr);
    sigaction(SIGBUS, &sa, nullptr);
}

uint64_t splitmix(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void die(const char *what, int rc) {
    std::fprintf(stderr, "%s failed: %d (%s)\n", what, rc, agn_last_error());
    std::exit(1);
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

struct Partition {
    agn_oplog *log = nullptr;
    agn_batcher *b = nullptr;
    std::vector<uint64_t> clock;                   // writer's copy
    std::unique_ptr<std::atomic<uint64_t>[]> pub;  // published clock (readers' R)
    std::vector<uint64_t> last;                    // set/register: last token per key x elem
    uint64_t tok = 1;
};

constexpr uint64_t NE = 16;  // set elements / register values per key

// One set/register effect of key k (writer state in pt): tag, add token and
// the tokens it removes / overrides.
void tag_effect(Partition &pt, uint32_t crdt, uint64_t k, uint64_t &seed, uint32_t &tag,
                uint64_t &add, std::vector<uint64_t> &rems) {
    const uint64_t e = splitmix(seed) % NE;
    tag = (uint32_t)e;
    add = pt.tok++;
    uint64_t &l = pt.last[crdt == AGN_SET_AW ? k * NE + e : k];
    if (l) rems.push_back(l);
    l = add;
}

}  // namespace

int main(int argc, char **argv) {
    uint64_t K = 250000, N = 64, D = 8, P = 1, T = 20, M = 5000, batch = 1024, wait = 0, hot = 0;
    uint64_t sparse = 0, present = 0, crash = 0;
    uint32_t crdt = AGN_COUNTER_PN;
    double wps = 0;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        const size_t eq = a.find('=');
        if (eq == std::string::npos) {
            std::fprintf(stderr, "bad argument %s (want name=value)\n", argv[i]);
            return 2;
        }
        const std::string k = a.substr(0, eq);
        const char *v = argv[i] + eq + 1;
        if (k == "keys") K = std::strtoull(v, nullptr, 10);
        else if (k == "ops") N = std::strtoull(v, nullptr, 10);
        else if (k == "dcs") D = std::strtoull(v, nullptr, 10);
        else if (k == "parts") P = std::strtoull(v, nullptr, 10);
        else if (k == "threads") T = std::strtoull(v, nullptr, 10);
        else if (k == "reads") M = std::strtoull(v, nullptr, 10);
        else if (k == "batch") batch = std::strtoull(v, nullptr, 10);
        else if (k == "wait") wait = std::strtoull(v, nullptr, 10);
        else if (k == "wps") wps = std::atof(v);
        else if (k == "hot") hot = std::strtoull(v, nullptr, 10);
        else if (k == "sparse") sparse = std::strtoull(v, nullptr, 10);
        else if (k == "present") present = std::strtoull(v, nullptr, 10);
        else if (k == "crash") crash = std::strtoull(v, nullptr, 10);
        else if (k == "type") {
            const std::string t = v;
            crdt = t == "set" ? AGN_SET_AW : t == "register" ? AGN_REGISTER_MV : AGN_COUNTER_PN;
            if (t != "set" && t != "register" && t != "counter") return 2;
        }
        else {
            std::fprintf(stderr, "unknown argument %s\n", argv[i]);
            return 2;
        }
    }
    if (present == 0) present = D;
    if (K == 0 || D == 0 || D > 64 || P == 0 || P > 64 || T == 0 || T * P > 1024 || present > D)
        return 2;
    // the interned DCs' presence word (sparse logs)
    const uint64_t pmask = present >= 64 ? ~0ull : ((1ull << present) - 1ull);
    const uint64_t H = (hot == 0 || hot > K) ? K : hot;  // keys read / written

    agn_ctx *ctx = nullptr;
    int rc = agn_open(0, &ctx);
    if (rc) die("agn_open", rc);
    if (crash) install_crash_handler();
    std::vector<Partition> parts(P);
    double t_load = now_s();
    for (uint64_t p = 0; p < P; ++p) {
        Partition &pt = parts[p];
        const bool tags = crdt != AGN_COUNTER_PN;
        if (tags) pt.last.assign(crdt == AGN_SET_AW ? K * NE : K, 0);
        if ((rc = agn_oplog_create(ctx, crdt, (uint32_t)D, K, (int)sparse, 0, &pt.log)))
            die("agn_oplog_create", rc);
        // the partition's history: N ops per key, commit clocks increasing per DC
        pt.clock.assign(D, 1700000000000000ull);
        uint64_t seed = 20250112ull + p;
        const uint64_t chunk = 1u << 20;
        std::vector<uint64_t> keys, oc, ocm, add, rem;
        std::vector<int64_t> eff;
        std::vector<uint32_t> tag, roff;
        for (uint64_t done = 0; done < K * N;) {
            const uint64_t n = std::min(chunk, K * N - done);
            keys.resize(n);
            oc.resize(n * D);
            eff.resize(n);
            ocm.assign(sparse ? n : 0, pmask);
            tag.resize(tags ? n : 0);
            add.resize(tags ? n : 0);
            roff.assign(tags ? n + 1 : 0, 0);
            rem.clear();
            for (uint64_t i = 0; i < n; ++i) {
                keys[i] = (done + i) % K;  // ops of keys interleave, as updates do
                const uint32_t dc = (uint32_t)(splitmix(seed) % present);
                pt.clock[dc] += 1 + splitmix(seed) % 1000;
                for (uint32_t d = 0; d < D; ++d) {
                    const uint64_t lag = splitmix(seed) % 5000;
                    const uint64_t c = pt.clock[d];
                    oc[i * D + d] = d >= present ? 0 : d == dc ? c : (c > lag ? c - lag : 0);
                }
                eff[i] = (int64_t)(splitmix(seed) % 2001) - 1000;
                if (tags) {
                    tag_effect(pt, crdt, keys[i], seed, tag[i], add[i], rem);
                    roff[i + 1] = (uint32_t)rem.size();
                }
            }
            if (tags && rem.empty()) rem.push_back(0);
            if ((rc = agn_oplog_append(pt.log, n, keys.data(), nullptr, oc.data(),
                                       sparse ? ocm.data() : nullptr, nullptr,
                                       tags ? nullptr : eff.data(), tags ? tag.data() : nullptr,
                                       tags ? add.data() : nullptr, tags ? roff.data() : nullptr,
                                       tags ? rem.data() : nullptr, nullptr, nullptr)))
                die("agn_oplog_append", rc);
            done += n;
        }
        pt.pub.reset(new std::atomic<uint64_t>[D]);
        for (uint64_t d = 0; d < D; ++d) pt.pub[d].store(pt.clock[d]);
        if ((rc = agn_batcher_create_cached(pt.log, 0, (uint32_t)batch, (uint32_t)wait, &pt.b)))
            die("agn_batcher_create_cached", rc);
    }
    t_load = now_s() - t_load;

    // R of a read: the partition's published clock (one writer, lock-free
    // readers; a reader may see some DCs one update newer than others -- still
    // a clock every op of the log is either inside of or not)
    auto snapshot_clock = [&](const Partition &pt, std::vector<uint64_t> &r) {
        r.resize(D);
        for (uint64_t d = 0; d < D; ++d) r[d] = pt.pub[d].load(std::memory_order_acquire);
    };
    // warm-up: the first 4096 keys of every partition once
    for (auto &pt : parts) {
        std::vector<uint64_t> R, ct(D), otok(4 * NE);
        std::vector<uint32_t> otag(4 * NE);
        uint64_t ctm = 0;
        snapshot_clock(pt, R);
        agn_key_read rd{};
        agn_key_result o{};
        rd.R = R.data();
        rd.R_mask = sparse ? &pmask : nullptr;
        o.lastct = ct.data();
        o.lastct_mask = sparse ? &ctm : nullptr;
        o.out_cap = (uint32_t)otag.size();
        o.out_tag = otag.data();
        o.out_tok = otok.data();
        for (uint64_t k = 0; k < std::min<uint64_t>(H, 4096); ++k) {
            rd.key = k;
            if ((rc = agn_batcher_read(pt.b, &rd, &o))) die("agn_batcher_read (warm-up)", rc);
        }
    }
    std::vector<uint64_t> b0(P), r0(P);
    for (uint64_t p = 0; p < P; ++p) agn_batcher_stats(parts[p].b, &b0[p], &r0[p]);

    std::atomic<bool> stop{false};
    std::atomic<uint64_t> writes{0};
    std::vector<std::thread> writers;
    if (wps > 0) {
        for (uint64_t p = 0; p < P; ++p) {
            writers.emplace_back([&, p] {
                Partition &pt = parts[p];
                uint64_t ws = 777 + p;
                const double dt = 1.0 / wps;
                double next = now_s();
                std::vector<uint64_t> row(D), rems;
                const bool tags = crdt != AGN_COUNTER_PN;
                while (!stop.load(std::memory_order_relaxed)) {
                    const uint64_t key = splitmix(ws) % H;
                    const uint32_t dc = (uint32_t)(splitmix(ws) % present);
                    pt.clock[dc] += 1 + splitmix(ws) % 1000;
                    for (uint64_t d = 0; d < D; ++d) row[d] = d < present ? pt.clock[d] : 0;
                    const int64_t e = (int64_t)(splitmix(ws) % 2001) - 1000;
                    uint32_t tg = 0, ro[2] = {0, 0};
                    uint64_t ad = 0;
                    rems.clear();
                    if (tags) tag_effect(pt, crdt, key, ws, tg, ad, rems);
                    ro[1] = (uint32_t)rems.size();
                    if (rems.empty()) rems.push_back(0);
                    if (agn_oplog_append(pt.log, 1, &key, nullptr, row.data(),
                                         sparse ? &pmask : nullptr, nullptr, tags ? nullptr : &e,
                                         tags ? &tg : nullptr, tags ? &ad : nullptr,
                                         tags ? ro : nullptr, tags ? rems.data() : nullptr, nullptr,
                                         nullptr))
                        die("agn_oplog_append (writer)", -1);
                    // published after the append: a read at the new clock sees the op
                    pt.pub[dc].store(pt.clock[dc], std::memory_order_release);
                    writes.fetch_add(1, std::memory_order_relaxed);
                    next += dt;
                    const double w = next - now_s();
                    if (w > 0) std::this_thread::sleep_for(std::chrono::duration<double>(w));
                }
            });
        }
    }

    const uint64_t NT = P * T;
    std::vector<std::vector<float>> lat(NT);
    std::vector<uint64_t> st_hit(NT), st_new(NT), st_log(NT), errs(NT);
    std::vector<std::thread> th;
    const double t0 = now_s();
    for (uint64_t t = 0; t < NT; ++t) {
        th.emplace_back([&, t] {
            Partition &pt = parts[t % P];
            uint64_t s = 1000 + t;
            std::vector<uint64_t> R, ct(D), otok(4 * NE);
            std::vector<uint32_t> otag(4 * NE);
            uint64_t ctm = 0;
            agn_key_read rd{};
            agn_key_result o{};
            o.lastct = ct.data();
            o.lastct_mask = sparse ? &ctm : nullptr;
            o.out_cap = (uint32_t)otag.size();
            o.out_tag = otag.data();
            o.out_tok = otok.data();
            rd.R_mask = sparse ? &pmask : nullptr;
            lat[t].reserve(M);
            for (uint64_t i = 0; i < M; ++i) {
                snapshot_clock(pt, R);
                rd.key = splitmix(s) % H;
                rd.R = R.data();
                const double a = now_s();
                const int r = agn_batcher_read(pt.b, &rd, &o);
                lat[t].push_back((float)((now_s() - a) * 1e6));
                if (r) {
                    ++errs[t];
                    continue;
                }
                if (o.status == AGN_SS_HIT) ++st_hit[t];
                else if (o.status == AGN_SS_NEW) ++st_new[t];
                else ++st_log[t];
            }
        });
    }
    for (auto &x : th) x.join();
    const double el = now_s() - t0;
    stop = true;
    for (auto &w : writers) w.join();

    uint64_t batches = 0, breads = 0;
    for (uint64_t p = 0; p < P; ++p) {
        uint64_t b1 = 0, r1 = 0;
        agn_batcher_stats(parts[p].b, &b1, &r1);
        batches += b1 - b0[p];
        breads += r1 - r0[p];
    }
    std::vector<float> all;
    for (auto &v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    auto pct = [&](double q) { return all.empty() ? 0.0 : (double)all[(size_t)(q * (all.size() - 1))]; };
    uint64_t hit = 0, nw = 0, lg = 0, er = 0;
    for (uint64_t t = 0; t < NT; ++t) {
        hit += st_hit[t];
        nw += st_new[t];
        lg += st_log[t];
        er += errs[t];
    }
    const uint64_t reads = NT * M;
    std::printf(
        "{\"tool\": \"serve_bench\", \"type\": \"%s\", \"log\": \"%s\", \"dcs_present\": %llu, "
        "\"parts\": %llu, \"keys_per_part\": %llu, \"hot_keys\": %llu, "
        "\"ops_per_key\": %llu, \"n_dcs\": %llu, \"threads_per_part\": %llu, \"reads\": %llu, "
        "\"max_batch\": %llu, \"max_wait_us\": %llu, \"writes_per_s_per_part\": %.0f, "
        "\"writes\": %llu, \"load_s\": %.3f, \"elapsed_s\": %.4f, \"reads_per_s\": %.1f, "
        "\"lat_us\": {\"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"max\": %.1f}, "
        "\"batches\": %llu, \"mean_batch\": %.2f, \"status\": {\"hit\": %llu, \"new\": %llu, "
        "\"log\": %llu}, \"errors\": %llu}\n",
        crdt == AGN_SET_AW ? "set_aw" : crdt == AGN_REGISTER_MV ? "register_mv" : "counter_pn",
        sparse ? "sparse (presence masks, as the NIF builds it)" : "dense", (unsigned long long)present,
        (unsigned long long)P, (unsigned long long)K, (unsigned long long)H, (unsigned long long)N,
        (unsigned long long)D, (unsigned long long)T, (unsigned long long)reads,
        (unsigned long long)batch, (unsigned long long)wait, wps,
        (unsigned long long)writes.load(), t_load, el, reads / el, pct(0.5), pct(0.9), pct(0.99),
        all.empty() ? 0.0 : (double)all.back(), (unsigned long long)batches,
        batches ? (double)breads / (double)batches : 0.0, (unsigned long long)hit,
        (unsigned long long)nw, (unsigned long long)lg, (unsigned long long)er);
    for (auto &pt : parts) {
        agn_batcher_destroy(pt.b);
        agn_oplog_destroy(pt.log);
    }
    agn_close(ctx);
    return er ? 1 : 0;
}
