// TEST INFRASTRUCTURE: a stand-in for librccl with the calls csrc/rs_mgpu.hip makes (ncclGetUniqueId,
// ncclCommInitRank, ncclCommSplit, ncclCommDestroy, ncclGroupStart / ncclGroupEnd, ncclSend / ncclRecv,
// ncclAllReduce, ncclGetErrorString), so that the RCCL branch of rs_mgpu (its NcclLink transfers, the per-lane
// communicators, the all-reduce of rs_mgpu_rebalance) runs with several ranks on ONE GPU: RCCL itself refuses
// two ranks on one device.  Ranks are threads of one process.  A send and a receive pair up by (communicator
// group, sender, receiver, issue order), as in NCCL; the pair becomes a hipMemcpyAsync on the receiver's stream
// after an event on the sender's stream (the data the send reads is complete), and the sender's stream then
// waits for the copy (its later work may overwrite the buffer).  Every group waits on the host until all of its
// operations are paired -- the checks: equal byte counts per pair, nothing left unpaired (timeout) -- and
// rccl_stub_stats() reports pairs, bytes, mismatches and all-reduces.  Linked only into
// tests/cpp/_build/librestir_rcclstub.so (tests/cpp/Makefile), never into the product.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <tuple>
#include <vector>

namespace {

struct Group;
std::mutex g_mu;
std::condition_variable g_cv;
long g_pairs = 0, g_bytes = 0, g_mismatch = 0, g_unpaired = 0, g_allreduce = 0;
std::vector<hipEvent_t> g_events;                 // destroyed when the last communicator goes

struct Op {
    bool send;
    const void* sbuf;
    void* rbuf;
    size_t bytes;
    int src, dst;
    hipStream_t st;
    hipEvent_t ready = nullptr, done = nullptr;
    bool paired = false, bad = false;
};

struct Group {
    int n = 0;
    int joined = 0;
    std::vector<int> split_seq;                   // per rank: splits called
    // split bookkeeping: (seq) -> per rank (color, key) and the resulting groups
    struct Split { int called = 0; std::vector<int> color, key; std::map<int, Group*> out; bool done = false; };
    std::map<int, Split> splits;
    std::map<std::pair<int, int>, std::deque<Op*>> sends, recvs;   // (src, dst)
    // all-reduce: per call sequence
    struct Red { int posted = 0; std::vector<std::vector<double>> in; std::vector<double> out; bool done = false; int dtype = 0, op = 0; };
    std::map<int, Red> reds;
    std::vector<int> red_seq;
};
std::map<std::string, Group*> g_registry;
int g_live_comms = 0;

hipEvent_t new_event() {
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    g_events.push_back(e);
    return e;
}

// under g_mu: pair queued sends and receives of (src, dst)
void try_pair(Group* g, std::pair<int, int> key) {
    auto& S = g->sends[key];
    auto& R = g->recvs[key];
    while (!S.empty() && !R.empty()) {
        Op* s = S.front();
        Op* r = R.front();
        S.pop_front();
        R.pop_front();
        s->paired = r->paired = true;
        if (s->bytes != r->bytes) {
            s->bad = r->bad = true;
            ++g_mismatch;
            std::fprintf(stderr, "rccl_stub: send %d->%d of %zu B paired with a receive of %zu B\n", s->src, s->dst, s->bytes,
                         r->bytes);
            continue;
        }
        hipEvent_t done = new_event();
        if (hipStreamWaitEvent(r->st, s->ready, 0) != hipSuccess ||
            hipMemcpyAsync(r->rbuf, s->sbuf, s->bytes, hipMemcpyDeviceToDevice, r->st) != hipSuccess || !done ||
            hipEventRecord(done, r->st) != hipSuccess) {
            s->bad = r->bad = true;
            continue;
        }
        s->done = r->done = done;
        ++g_pairs;
        g_bytes += (long)s->bytes;
    }
}

thread_local int t_depth = 0;
thread_local std::vector<Op*> t_ops;
thread_local std::vector<Group*> t_op_group;

ncclResult_t finish_ops() {
    std::vector<Op*> ops;
    std::vector<Group*> grp;
    ops.swap(t_ops);
    grp.swap(t_op_group);
    {
        std::unique_lock<std::mutex> lk(g_mu);
        for (size_t i = 0; i < ops.size(); ++i) {
            Op* o = ops[i];
            o->ready = new_event();
            if (!o->ready || hipEventRecord(o->ready, o->st) != hipSuccess) return ncclUnhandledCudaError;
            const std::pair<int, int> key{o->src, o->dst};
            (o->send ? grp[i]->sends : grp[i]->recvs)[key].push_back(o);
            try_pair(grp[i], key);
        }
        g_cv.notify_all();
        const bool ok = g_cv.wait_for(lk, std::chrono::seconds(60), [&] {
            for (Op* o : ops) if (!o->paired) return false;
            return true;
        });
        if (!ok) {
            g_unpaired += 1;
            std::fprintf(stderr, "rccl_stub: a group's operations stayed unpaired for 60 s\n");
            return ncclInternalError;
        }
    }
    ncclResult_t rc = ncclSuccess;
    for (Op* o : ops) {
        if (o->bad) rc = ncclInvalidUsage;
        else if (o->send && hipStreamWaitEvent(o->st, o->done, 0) != hipSuccess) rc = ncclUnhandledCudaError;
        delete o;
    }
    return rc;
}

ncclResult_t post(bool send, const void* sb, void* rb, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm,
                  hipStream_t st);

}  // namespace

struct ncclComm {
    Group* g;
    int rank;
};

namespace {
size_t dtype_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        default: return 8;
    }
}
ncclResult_t post(bool send, const void* sb, void* rb, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm,
                  hipStream_t st) {
    if (!comm || peer < 0 || peer >= comm->g->n || peer == comm->rank) return ncclInvalidArgument;
    Op* o = new Op{send, sb, rb, count * dtype_bytes(dt), send ? comm->rank : peer, send ? peer : comm->rank, st};
    t_ops.push_back(o);
    t_op_group.push_back(comm->g);
    return t_depth == 0 ? finish_ops() : ncclSuccess;
}
}  // namespace

extern "C" {

void rccl_stub_stats(long* pairs, long* bytes, long* mismatches, long* unpaired, long* allreduces) {
    std::lock_guard<std::mutex> lk(g_mu);
    *pairs = g_pairs; *bytes = g_bytes; *mismatches = g_mismatch; *unpaired = g_unpaired; *allreduces = g_allreduce;
}

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (rccl_stub)";
        case ncclInvalidArgument: return "invalid argument (rccl_stub)";
        case ncclInvalidUsage: return "invalid usage: paired byte counts differ (rccl_stub)";
        case ncclInternalError: return "unpaired operations (rccl_stub)";
        default: return "error (rccl_stub)";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    static std::mt19937_64 rng(std::random_device{}());
    std::lock_guard<std::mutex> lk(g_mu);
    std::memset(id->internal, 0, sizeof id->internal);
    const uint64_t v[2] = {rng(), rng()};
    std::memcpy(id->internal, v, sizeof v);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    std::unique_lock<std::mutex> lk(g_mu);
    const std::string key(id.internal, sizeof id.internal);
    Group*& g = g_registry[key];
    if (!g) { g = new Group(); g->n = nranks; g->split_seq.assign(nranks, 0); g->red_seq.assign(nranks, 0); }
    if (g->n != nranks) return ncclInvalidArgument;
    ++g->joined;
    g_cv.notify_all();
    Group* gg = g;
    if (!g_cv.wait_for(lk, std::chrono::seconds(60), [&] { return gg->joined >= gg->n; })) return ncclInternalError;
    *comm = new ncclComm{gg, rank};
    ++g_live_comms;
    return ncclSuccess;
}

ncclResult_t ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm, ncclConfig_t*) {
    if (!comm || !newcomm) return ncclInvalidArgument;
    std::unique_lock<std::mutex> lk(g_mu);
    Group* g = comm->g;
    const int seq = g->split_seq[comm->rank]++;
    Group::Split& S = g->splits[seq];
    if (S.color.empty()) { S.color.assign(g->n, -1); S.key.assign(g->n, 0); }
    S.color[comm->rank] = color;
    S.key[comm->rank] = key;
    if (++S.called == g->n) {                       // everybody is here: form the groups
        std::map<int, std::vector<std::pair<int, int>>> by;   // color -> (key, parent rank)
        for (int r = 0; r < g->n; ++r) if (S.color[r] >= 0) by[S.color[r]].push_back({S.key[r], r});
        for (auto& kv : by) {
            Group* ng = new Group();
            ng->n = (int)kv.second.size();
            ng->joined = ng->n;
            ng->split_seq.assign(ng->n, 0);
            ng->red_seq.assign(ng->n, 0);
            S.out[kv.first] = ng;
        }
        S.done = true;
        g_cv.notify_all();
    }
    if (!g_cv.wait_for(lk, std::chrono::seconds(60), [&] { return S.done; })) return ncclInternalError;
    if (color < 0) { *newcomm = nullptr; return ncclSuccess; }
    std::vector<std::pair<int, int>> mem;
    for (int r = 0; r < g->n; ++r) if (S.color[r] == color) mem.push_back({S.key[r], r});
    std::sort(mem.begin(), mem.end());
    int nr = 0;
    while (mem[nr].second != comm->rank) ++nr;
    *newcomm = new ncclComm{S.out[color], nr};
    ++g_live_comms;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return ncclSuccess;
    std::lock_guard<std::mutex> lk(g_mu);
    delete comm;
    if (--g_live_comms == 0) {
        (void)hipDeviceSynchronize();
        for (hipEvent_t e : g_events) (void)hipEventDestroy(e);
        g_events.clear();
    }
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() { ++t_depth; return ncclSuccess; }
ncclResult_t ncclGroupEnd() {
    if (t_depth <= 0) return ncclInvalidUsage;
    return --t_depth == 0 ? finish_ops() : ncclSuccess;
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm, hipStream_t stream) {
    return post(true, sendbuff, nullptr, count, datatype, peer, comm, stream);
}
ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm, hipStream_t stream) {
    return post(false, nullptr, recvbuff, count, datatype, peer, comm, stream);
}

// host-synchronous all-reduce of float64 / float32 values (sum or max; ranks combined in rank order)
ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream) {
    if (!comm || (datatype != ncclFloat64 && datatype != ncclFloat32) || (op != ncclSum && op != ncclMax)) return ncclInvalidArgument;
    const size_t eb = dtype_bytes(datatype);
    std::vector<char> raw(count * eb);
    if (hipMemcpyAsync(raw.data(), sendbuff, raw.size(), hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
    std::vector<double> v(count);
    for (size_t i = 0; i < count; ++i) {
        if (datatype == ncclFloat64) std::memcpy(&v[i], &raw[8 * i], 8);
        else { float f; std::memcpy(&f, &raw[4 * i], 4); v[i] = f; }
    }
    std::vector<double> out;
    {
        std::unique_lock<std::mutex> lk(g_mu);
        Group* g = comm->g;
        const int seq = g->red_seq[comm->rank]++;
        Group::Red& R = g->reds[seq];
        if (R.in.empty()) R.in.resize(g->n);
        R.in[comm->rank] = v;
        if (++R.posted == g->n) {
            R.out = R.in[0];
            for (int r = 1; r < g->n; ++r)
                for (size_t i = 0; i < count; ++i)
                    R.out[i] = op == ncclSum ? R.out[i] + R.in[r][i] : (R.in[r][i] > R.out[i] ? R.in[r][i] : R.out[i]);
            R.done = true;
            ++g_allreduce;
            g_cv.notify_all();
        }
        if (!g_cv.wait_for(lk, std::chrono::seconds(60), [&] { return R.done; })) return ncclInternalError;
        out = R.out;
    }
    for (size_t i = 0; i < count; ++i) {
        if (datatype == ncclFloat64) std::memcpy(&raw[8 * i], &out[i], 8);
        else { const float f = (float)out[i]; std::memcpy(&raw[4 * i], &f, 4); }
    }
    if (hipMemcpyAsync(recvbuff, raw.data(), raw.size(), hipMemcpyHostToDevice, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
    return ncclSuccess;
}

}  // extern "C"
