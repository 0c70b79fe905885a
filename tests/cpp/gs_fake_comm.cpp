// gs_fake_comm.cpp -- TEST INFRASTRUCTURE: an in-process emulation of the collectives a
// gs_group uses (include/gs_group.h, gs_comm_api), installed with
// gs_group_set_comm_api(gs_fake_comm_api()). N threads of ONE process, each driving one
// rank's summary on the same GPU, meet at host barriers; the data moves with device
// copies ordered by events. RCCL refuses two ranks on one GPU and the GPU box has one,
// so this runs the group's N-rank code paths -- count and data all-gathers, the
// partitioned mode's all-to-all, the binomial tree's send/recv -- exactly as RCCL would
// be driven. Built into gelly-streaming_amd/host/bin/libgs_fakecomm.so (host Makefile);
// never loaded by the product path.
//
// Collective order check. Every rank thread keeps a running hash of
// the (communicator, call number) sequence of the collectives it has issued on all of
// its communicators. Each collective deposits that hash at its first barrier; if the
// ranks' hashes differ -- the ranks issued the same collectives in different
// interleavings across communicators, the condition that deadlocked the eager data
// halves of round 5 (0b5eb08) -- the call fails with "collective order differs". A
// barrier that waits more than 20 s fails the same way (an order that cannot meet).
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gs_group.h"

namespace {

constexpr int kIdBytes = 128;
constexpr int kErrOrder = 90, kErrTimeout = 91, kErrHip = 92, kErrSize = 93;

struct Shared {
  int n = 0, refs = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  std::vector<const void*> src;
  std::vector<hipEvent_t> ev;
  std::vector<uint64_t> sig;  // each rank's order hash at this collective
  // all-to-all: each rank's send buffer, counts and displacements (elements)
  std::vector<const size_t*> a2a_sc, a2a_sd;
  size_t elem = 8;
  struct Msg {
    const void* buf;
    size_t bytes;
    hipEvent_t ready, copied;
    bool done = false;
  };
  std::map<std::pair<int, int>, std::deque<Msg*>> box;  // (from, to) -> messages
};
struct Comm {
  Shared* s;
  int rank;
  uint64_t calls = 0;  // collectives issued on this communicator
  hipEvent_t ready = nullptr, done = nullptr;
  std::vector<hipEvent_t> spare;  // message events, destroyed with the comm
};
std::mutex g_mu;
std::map<std::string, Shared*> g_reg;
thread_local uint64_t t_order = 0x9E3779B97F4A7C15ull;  // this rank thread's order hash
std::atomic<int> g_last_err{0};
std::atomic<int> g_timeout_ms{20000};  // a collective's ranks must meet within this

// Serialized replay (gs_fake_comm_set_serialize): a rank thread holds the GPU token
// whenever it is outside a collective, so the ranks' work between two collectives runs
// one rank at a time and each rank's HIP events time its own work alone (tools/part_replay.py:
// the per-rank cost of an N-GPU pass, measured on one GPU).
std::atomic<bool> g_serialize{false};
std::mutex g_token;
thread_local bool t_token = false;
void token_release() {
  if (g_serialize && t_token) {
    // this rank's queued device work (every stream) finishes before another rank runs: the
    // other ranks are idle (they synchronised when they released the token)
    (void)hipDeviceSynchronize();
    t_token = false;
    g_token.unlock();
  }
}
void token_acquire() {
  if (g_serialize && !t_token) {
    g_token.lock();
    t_token = true;
  }
}
struct TokenGap {  // inside a collective: the token is free for the other ranks
  TokenGap() { token_release(); }
  ~TokenGap() { token_acquire(); }
};

uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

int barrier(Shared* s) {
  std::unique_lock<std::mutex> lk(s->m);
  const uint64_t g0 = s->gen;
  if (++s->arrived == s->n) {
    s->arrived = 0;
    s->gen++;
    s->cv.notify_all();
    return 0;
  }
  if (!s->cv.wait_for(lk, std::chrono::milliseconds(g_timeout_ms.load()), [&] { return s->gen != g0; })) {
    --s->arrived;
    return kErrTimeout;
  }
  return 0;
}

// The collective's first meeting: record this rank's order hash, check every rank's.
int order_check(Comm* c) {
  Shared* s = c->s;
  t_order = mix(t_order ^ (reinterpret_cast<uintptr_t>(s) * 0x100000001B3ull + c->calls++));
  {
    std::lock_guard<std::mutex> lk(s->m);
    s->sig[c->rank] = t_order;
  }
  if (int e = barrier(s)) return e;
  int rc = 0;
  {
    std::lock_guard<std::mutex> lk(s->m);
    for (int q = 0; q < s->n; ++q)
      if (s->sig[q] != s->sig[c->rank]) rc = kErrOrder;
  }
  return rc;
}

size_t elem(int dtype) { return dtype == 1 ? 1 : 8; }

int f_unique_id(void* id) {
  static std::atomic<uint64_t> ctr{1};
  memset(id, 0, kIdBytes);
  const uint64_t v[2] = {(uint64_t)getpid(), ctr++};
  memcpy(id, v, sizeof v);
  return 0;
}
int f_init(void** comm, int n, const void* id, int rank) {
  std::lock_guard<std::mutex> lk(g_mu);
  Shared*& s = g_reg[std::string(static_cast<const char*>(id), kIdBytes)];
  if (!s) {
    s = new Shared();
    s->n = n;
    s->src.resize(n);
    s->ev.resize(n);
    s->sig.resize(n);
    s->a2a_sc.resize(n);
    s->a2a_sd.resize(n);
  }
  s->refs++;
  Comm* c = new Comm{s, rank};
  t_order = 0x9E3779B97F4A7C15ull;  // every rank creates its communicators in one order
  if (hipEventCreateWithFlags(&c->ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess)
    return kErrHip;
  *comm = c;
  return 0;
}
int f_destroy(void* comm) {
  Comm* c = (Comm*)comm;
  (void)hipEventDestroy(c->ready);
  (void)hipEventDestroy(c->done);
  for (hipEvent_t e : c->spare) (void)hipEventDestroy(e);
  std::lock_guard<std::mutex> lk(g_mu);
  if (--c->s->refs == 0) {
    for (auto it = g_reg.begin(); it != g_reg.end(); ++it)
      if (it->second == c->s) {
        g_reg.erase(it);
        break;
      }
    delete c->s;
  }
  delete c;
  return 0;
}
// After the copies: every rank waits (on its stream) until every other rank has read
// its send buffer, then the slots may be reused.
int finish_collective(Comm* c, hipStream_t st) {
  Shared* s = c->s;
  if (hipEventRecord(c->done, st) != hipSuccess) return kErrHip;
  if (int e = barrier(s)) return e;  // (the ready events were captured by every stream's wait)
  {
    std::lock_guard<std::mutex> lk(s->m);
    s->ev[c->rank] = c->done;
  }
  if (int e = barrier(s)) return e;
  for (int q = 0; q < s->n; ++q)
    if (q != c->rank && hipStreamWaitEvent(st, s->ev[q], 0) != hipSuccess) return kErrHip;
  return barrier(s);
}
int f_all_gather(const void* send, void* recv, size_t count, int dtype, void* comm, void* stream) {
  TokenGap gap;
  Comm* c = (Comm*)comm;
  Shared* s = c->s;
  hipStream_t st = (hipStream_t)stream;
  const size_t bytes = count * elem(dtype);
  if (int e = order_check(c)) return g_last_err = e;
  if (hipEventRecord(c->ready, st) != hipSuccess) return kErrHip;
  {
    std::lock_guard<std::mutex> lk(s->m);
    s->src[c->rank] = send;
    s->ev[c->rank] = c->ready;
  }
  if (int e = barrier(s)) return g_last_err = e;  // every rank's send buffer is staged (in its stream order)
  for (int q = 0; q < s->n; ++q) {
    if (hipStreamWaitEvent(st, s->ev[q], 0) != hipSuccess) return kErrHip;
    if (bytes && hipMemcpyAsync((char*)recv + (size_t)q * bytes, s->src[q], bytes, hipMemcpyDeviceToDevice, st) !=
                     hipSuccess)
      return kErrHip;
  }
  // serialized replay: the collective's copies are done on every rank before any rank runs on
  if (g_serialize && hipStreamSynchronize(st) != hipSuccess) return kErrHip;
  if (int e = finish_collective(c, st)) return g_last_err = e;
  return 0;
}
int f_all_to_allv(const void* send, const size_t* sc, const size_t* sd, void* recv, const size_t* rc,
                  const size_t* rd, int dtype, void* comm, void* stream) {
  TokenGap gap;
  Comm* c = (Comm*)comm;
  Shared* s = c->s;
  hipStream_t st = (hipStream_t)stream;
  const size_t es = elem(dtype);
  if (int e = order_check(c)) return g_last_err = e;
  if (hipEventRecord(c->ready, st) != hipSuccess) return kErrHip;
  {
    std::lock_guard<std::mutex> lk(s->m);
    s->src[c->rank] = send;
    s->ev[c->rank] = c->ready;
    s->a2a_sc[c->rank] = sc;
    s->a2a_sd[c->rank] = sd;
  }
  if (int e = barrier(s)) return g_last_err = e;
  for (int q = 0; q < s->n; ++q) {  // block q -> this rank: q's send block for this rank
    const size_t n = s->a2a_sc[q][c->rank];
    if (n != rc[q]) return g_last_err = kErrSize;
    if (hipStreamWaitEvent(st, s->ev[q], 0) != hipSuccess) return kErrHip;
    if (n && hipMemcpyAsync((char*)recv + rd[q] * es, (const char*)s->src[q] + s->a2a_sd[q][c->rank] * es, n * es,
                            hipMemcpyDeviceToDevice, st) != hipSuccess)
      return kErrHip;
  }
  // serialized replay: the collective's copies are done on every rank before any rank runs on
  if (g_serialize && hipStreamSynchronize(st) != hipSuccess) return kErrHip;
  if (int e = finish_collective(c, st)) return g_last_err = e;
  return 0;
}
// point-to-point: not part of the order hash (a tree's ranks legitimately issue
// different send/recv sequences)
int f_send(const void* buf, size_t count, int dtype, int peer, void* comm, void* stream) {
  TokenGap gap;
  Comm* c = (Comm*)comm;
  Shared* s = c->s;
  hipStream_t st = (hipStream_t)stream;
  Shared::Msg msg{buf, count * elem(dtype), nullptr, nullptr};
  if (hipEventCreateWithFlags(&msg.ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&msg.copied, hipEventDisableTiming) != hipSuccess || hipEventRecord(msg.ready, st))
    return kErrHip;
  c->spare.push_back(msg.ready);
  c->spare.push_back(msg.copied);
  std::unique_lock<std::mutex> lk(s->m);
  s->box[{c->rank, peer}].push_back(&msg);
  s->cv.notify_all();
  if (!s->cv.wait_for(lk, std::chrono::seconds(20), [&] { return msg.done; })) return g_last_err = kErrTimeout;
  return hipStreamWaitEvent(st, msg.copied, 0) == hipSuccess ? 0 : kErrHip;
}
int f_recv(void* buf, size_t count, int dtype, int peer, void* comm, void* stream) {
  TokenGap gap;
  Comm* c = (Comm*)comm;
  Shared* s = c->s;
  hipStream_t st = (hipStream_t)stream;
  std::unique_lock<std::mutex> lk(s->m);
  auto& q = s->box[{peer, c->rank}];
  if (!s->cv.wait_for(lk, std::chrono::seconds(20), [&] { return !q.empty(); })) return g_last_err = kErrTimeout;
  Shared::Msg* msg = q.front();
  q.pop_front();
  int r = 0;
  if (msg->bytes != count * elem(dtype)) r = kErrSize;
  if (!r && (hipStreamWaitEvent(st, msg->ready, 0) != hipSuccess ||
             hipMemcpyAsync(buf, msg->buf, msg->bytes, hipMemcpyDeviceToDevice, st) != hipSuccess ||
             hipEventRecord(msg->copied, st) != hipSuccess))
    r = kErrHip;
  msg->done = true;
  s->cv.notify_all();
  return r;
}
int f_count(void* comm, int* n) {
  *n = ((Comm*)comm)->s->n;
  return 0;
}
int f_noop() { return 0; }
const char* f_error(int e) {
  switch (e) {
    case kErrOrder:
      return "comm emulation: collective order differs between ranks (another interleaving of the "
             "communicators' collectives on some rank)";
    case kErrTimeout:
      return "comm emulation: a collective's ranks did not meet within 20 s (collective order differs)";
    case kErrSize:
      return "comm emulation: send and receive sizes differ";
    default:
      return "comm emulation: HIP call failed";
  }
}

const gs_comm_api g_api = {f_unique_id, f_init,  f_destroy, f_count,  f_all_gather, f_all_to_allv,
                           f_send,      f_recv,  f_noop,    f_noop,   f_error};

}  // namespace

extern "C" {
const gs_comm_api* gs_fake_comm_api(void) { return &g_api; }
// the last order / timeout / size error any rank hit (0: none), then cleared
int gs_fake_comm_last_error(void) { return g_last_err.exchange(0); }
// the calling thread's order hash (tests compare ranks' hashes after a run)
uint64_t gs_fake_comm_order_hash(void) { return t_order; }
void gs_fake_comm_reset_order(void) { t_order = 0x9E3779B97F4A7C15ull; }
// serialized replay: on -> every rank thread must call gs_fake_comm_token(1) before its first
// GPU work and gs_fake_comm_token(0) when it is done
void gs_fake_comm_set_serialize(int on) { g_serialize = on != 0; }
void gs_fake_comm_token(int take) {
  if (take) token_acquire();
  else token_release();
}
// Self-test of the order check (tests/test_gpu_group_emulated.py): two rank threads join two
// communicators C and D and issue one empty all-gather on each -- rank 1 in the other order
// when `misorder`. errs[2 * r + k] = rank r's k-th collective result (misordered: each rank
// waits on the communicator the other rank is not in, kErrTimeout after timeout_ms, or
// kErrOrder where they meet with different histories; in order: 0).
int gs_fake_comm_selftest(int misorder, int timeout_ms, int* errs) {
  const int saved = g_timeout_ms.exchange(timeout_ms);
  char idc[kIdBytes], idd[kIdBytes];
  f_unique_id(idc);
  f_unique_id(idd);
  auto rank = [&](int r) {
    void *c = nullptr, *d = nullptr;
    if (f_init(&c, 2, idc, r) || f_init(&d, 2, idd, r)) {
      errs[2 * r] = errs[2 * r + 1] = kErrHip;
      return;
    }
    void* first = (misorder && r == 1) ? d : c;
    void* second = first == c ? d : c;
    errs[2 * r] = f_all_gather(nullptr, nullptr, 0, 1, first, nullptr);
    errs[2 * r + 1] = f_all_gather(nullptr, nullptr, 0, 1, second, nullptr);
    (void)hipStreamSynchronize(nullptr);
    f_destroy(c);
    f_destroy(d);
  };
  std::thread t0(rank, 0), t1(rank, 1);
  t0.join();
  t1.join();
  g_timeout_ms = saved;
  g_last_err = 0;
  return 0;
}
}
