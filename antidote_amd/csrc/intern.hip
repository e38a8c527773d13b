// intern.hip — exact term interning for the Erlang binding (host code).
//
// The device op log stores every Erlang term it needs to compare or hand
// back as an integer: DC ids (clock columns), keys (segments), TxIds
// (is_op_in_snapshot's `TxId == Op#clocksi_payload.txid`,
// src/clocksi_materializer.erl:220), set elements / register values (tags)
// and tokens.  The NIF maps a term through its external term format
// (enif_term_to_binary): equal bytes <=> equal id, with no hashing shortcut
// -- the map compares the full byte strings, so distinct terms never share
// an id (the round-1 shim's 31-bit phash2 could).  Ids are dense from
// `first_id`; the reverse map hands the stored bytes back for decoding
// (enif_binary_to_term).  Readers take the table shared, inserts exclusive.
#include <deque>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <unordered_map>

#include "common.hpp"

struct agn_interner {
    uint64_t first_id = 1, max_ids = 0;
    mutable std::shared_mutex mu;
    std::deque<std::string> bytes;  // id - first_id -> term bytes (stable storage)
    std::unordered_map<std::string_view, uint64_t> ids;  // views into `bytes`
};

using namespace agn;

extern "C" {

int agn_interner_create(uint64_t first_id, uint64_t max_ids, agn_interner **out) {
    if (!out) return fail(AGN_EINVAL, "interner_create: null out");
    *out = nullptr;
    if (max_ids == 0 || first_id + max_ids < first_id)
        return fail(AGN_EINVAL, "interner_create: bad id range");
    agn_interner *t = new (std::nothrow) agn_interner;
    if (!t) return fail(AGN_ENOMEM, "interner_create");
    t->first_id = first_id;
    t->max_ids = max_ids;
    *out = t;
    return AGN_OK;
}

int agn_interner_destroy(agn_interner *t) {
    delete t;
    return AGN_OK;
}

int agn_intern(agn_interner *t, const void *data, size_t n, uint64_t *id, int *is_new) {
    if (!t || !id || (n && !data)) return fail(AGN_EINVAL, "intern: null argument");
    const std::string_view key((const char *)data, n);
    if (is_new) *is_new = 0;
    {
        std::shared_lock<std::shared_mutex> r(t->mu);
        auto it = t->ids.find(key);
        if (it != t->ids.end()) {
            *id = it->second;
            return AGN_OK;
        }
    }
    std::unique_lock<std::shared_mutex> w(t->mu);
    auto it = t->ids.find(key);  // another thread may have inserted it meanwhile
    if (it != t->ids.end()) {
        *id = it->second;
        return AGN_OK;
    }
    if (t->bytes.size() >= t->max_ids)
        return fail(AGN_ECAPACITY, "intern: table full (%llu ids)", (unsigned long long)t->max_ids);
    try {
        t->bytes.emplace_back(key);
        const uint64_t v = t->first_id + (t->bytes.size() - 1);
        t->ids.emplace(std::string_view(t->bytes.back()), v);
        *id = v;
    } catch (const std::bad_alloc &) {
        if (t->bytes.size() > t->ids.size()) t->bytes.pop_back();
        return fail(AGN_ENOMEM, "intern: insert");
    }
    if (is_new) *is_new = 1;
    return AGN_OK;
}

int agn_intern_find(const agn_interner *t, const void *data, size_t n, uint64_t *id, int *found) {
    if (!t || !id || !found || (n && !data)) return fail(AGN_EINVAL, "intern_find: null argument");
    std::shared_lock<std::shared_mutex> r(t->mu);
    auto it = t->ids.find(std::string_view((const char *)data, n));
    *found = it != t->ids.end();
    *id = *found ? it->second : 0;
    return AGN_OK;
}

int agn_intern_bytes(const agn_interner *t, uint64_t id, const void **data, size_t *n) {
    if (!t || !data || !n) return fail(AGN_EINVAL, "intern_bytes: null argument");
    std::shared_lock<std::shared_mutex> r(t->mu);
    if (id < t->first_id || id - t->first_id >= t->bytes.size())
        return fail(AGN_EINVAL, "intern_bytes: unknown id %llu", (unsigned long long)id);
    const std::string &s = t->bytes[id - t->first_id];  // deque: stable until destroy
    *data = s.data();
    *n = s.size();
    return AGN_OK;
}

int agn_interner_size(const agn_interner *t, uint64_t *n) {
    if (!t || !n) return fail(AGN_EINVAL, "interner_size: null argument");
    std::shared_lock<std::shared_mutex> r(t->mu);
    *n = t->bytes.size();
    return AGN_OK;
}

}  // extern "C"
