// Could a synchronous host-buffer call (one JNI encodeBulk / decodeBulk of an
// RS(10,4) 1 MiB-cell stripe) skip the staging copies? Instead of copying the
// caller's pageable rows into pinned staging and its outputs back, register
// the rows' pages with HIP for the call (hipHostRegister, mapped) and let the
// zero-copy kernel read and write them across the host link directly.
// The rows sit as a JVM lays out 1 MiB byte[]s: G1 allocates such humongous
// objects at the start of their own region, so each row's data begins 16
// bytes (the array header) past a 2 MiB boundary. Two registration shapes:
// one range covering every row, and one registration per row (what a library
// call does with rows from unrelated objects).
// Per call, in one process, interleaved:
//   staged      hrs_encode / hrs_decode (the product's current path)
//   registered  register the covering pages + hrs_*_dev over the host
//               pointers + sync + unregister
//   resident    the same kernels with the pages registered once (lower bound)
// Every variant's outputs are compared with the staged call's.
// Usage: register_zc_probe [calls]   (one JSON line)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/hrs.h"

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int calls = argc > 1 ? atoi(argv[1]) : 100;
  const int k = 10, p = 4, n = k + p;
  const size_t L = 1 << 20, gap = 16;
  hrs_opts o{};
  o.device = 0;
  hrs_codec* c = nullptr;
  if (hrs_create(k, p, &o, &c) != HRS_OK) return 1;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  // heap-like buffer: rows [0, n) then one repaired row, each 16 bytes into its own 2 MiB region
  const size_t region = 2u << 20;
  const size_t span = (n + 1) * region;
  uint8_t* heap = static_cast<uint8_t*>(aligned_alloc(region, span));
  std::vector<uint8_t*> row(n + 1);
  for (int r = 0; r <= n; ++r) row[r] = heap + r * region + gap;
  uint64_t z = 0x9E3779B97F4A7C15ull;
  for (int r = p; r < n; ++r)
    for (size_t i = 0; i < L; i += 8) {
      z ^= z << 13, z ^= z >> 7, z ^= z << 17;
      memcpy(row[r] + i, &z, 8);
    }
  std::vector<const uint8_t*> in(k);
  std::vector<uint8_t*> par(p);
  for (int i = 0; i < k; ++i) in[i] = row[p + i];
  for (int r = 0; r < p; ++r) par[r] = row[r];
  // staged reference outputs
  if (hrs_encode(c, in.data(), par.data(), L) != HRS_OK) return 2;
  std::vector<std::vector<uint8_t>> ref(p);
  for (int r = 0; r < p; ++r) ref[r].assign(par[r], par[r] + L);
  const int erased[1] = {p};
  int to_read[16];
  if (hrs_locations_to_read(c, erased, 1, to_read) != HRS_OK) return 2;
  std::sort(to_read, to_read + k);
  std::vector<int> ntr;
  for (int l = 0; l < n; ++l)
    if (!std::binary_search(to_read, to_read + k, l)) ntr.push_back(l);
  std::vector<const uint8_t*> reads(n, nullptr);
  for (int i = 0; i < k; ++i) reads[to_read[i]] = row[to_read[i]];
  uint8_t* lost = row[n];

  const uintptr_t a0 = reinterpret_cast<uintptr_t>(heap) & ~uintptr_t(4095);
  const uintptr_t a1 = (reinterpret_cast<uintptr_t>(heap) + span + 4095) & ~uintptr_t(4095);
  bool ok = true, same_addr = true;
  auto reg = [&]() {
    hipError_t e = hipHostRegister(reinterpret_cast<void*>(a0), a1 - a0, hipHostRegisterMapped);
    if (e != hipSuccess) {
      fprintf(stderr, "hipHostRegister: %s\n", hipGetErrorString(e));
      ok = false;
      return;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, reinterpret_cast<void*>(a0), 0) != hipSuccess || d != reinterpret_cast<void*>(a0))
      same_addr = false;
  };
  auto unreg = [&]() { (void)hipHostUnregister(reinterpret_cast<void*>(a0)); };
  // one registration per row: the pages under [row, row + L)
  auto reg_rows = [&]() {
    for (int r = 0; r <= n; ++r) {
      const uintptr_t b0 = reinterpret_cast<uintptr_t>(row[r]) & ~uintptr_t(4095);
      const uintptr_t b1 = (reinterpret_cast<uintptr_t>(row[r]) + L + 4095) & ~uintptr_t(4095);
      if (hipHostRegister(reinterpret_cast<void*>(b0), b1 - b0, hipHostRegisterMapped) != hipSuccess) ok = false;
    }
  };
  auto unreg_rows = [&]() {
    for (int r = 0; r <= n; ++r)
      (void)hipHostUnregister(reinterpret_cast<void*>(reinterpret_cast<uintptr_t>(row[r]) & ~uintptr_t(4095)));
  };
  auto enc_dev = [&]() {
    ok &= hrs_encode_dev(c, in.data(), 0, par.data(), 0, L, 1, s) == HRS_OK;
    ok &= hipStreamSynchronize(s) == hipSuccess;
  };
  auto dec_dev = [&]() {
    ok &= hrs_decode_dev(c, reads.data(), 0, &lost, 0, erased, 1, ntr.data(), static_cast<int>(ntr.size()), L, 1, s) ==
          HRS_OK;
    ok &= hipStreamSynchronize(s) == hipSuccess;
  };
  auto check = [&](const char* what) {
    for (int r = 0; r < p; ++r)
      if (memcmp(par[r], ref[r].data(), L) != 0) {
        fprintf(stderr, "%s: parity %d differs\n", what, r);
        ok = false;
      }
    if (memcmp(lost, row[p], L) != 0) {
      fprintf(stderr, "%s: repaired row differs\n", what);
      ok = false;
    }
  };
  double t_stage_enc = 0, t_stage_dec = 0, t_reg_enc = 0, t_reg_dec = 0, t_res_enc = 0, t_res_dec = 0, t_reg = 0,
         t_unreg = 0, t_rows_enc = 0, t_rows_dec = 0;
  for (int it = -3; it < calls; ++it) {
    const bool timed = it >= 0;
    for (int r = 0; r < p; ++r) memset(par[r], 0, L);
    memset(lost, 0, L);
    double t0 = now_us();
    ok &= hrs_encode(c, in.data(), par.data(), L) == HRS_OK;
    double t1 = now_us();
    ok &= hrs_decode(c, reads.data(), &lost, erased, 1, to_read, k, ntr.data(), static_cast<int>(ntr.size()), L) ==
          HRS_OK;
    double t2 = now_us();
    if (it == 0) check("staged");
    for (int r = 0; r < p; ++r) memset(par[r], 0, L);
    memset(lost, 0, L);
    double t3 = now_us();
    reg();
    double t4 = now_us();
    enc_dev();
    double t5 = now_us();
    unreg();
    double t6 = now_us();
    reg();
    dec_dev();
    unreg();
    double t7 = now_us();
    if (it == 0) check("registered");
    for (int r = 0; r < p; ++r) memset(par[r], 0, L);
    memset(lost, 0, L);
    double t8 = now_us();
    reg_rows();
    enc_dev();
    unreg_rows();
    double t9 = now_us();
    reg_rows();
    dec_dev();
    unreg_rows();
    double t10 = now_us();
    if (it == 0) check("registered per row");
    if (timed) {
      t_rows_enc += t9 - t8;
      t_rows_dec += t10 - t9;
      t_stage_enc += t1 - t0;
      t_stage_dec += t2 - t1;
      t_reg_enc += t6 - t3;
      t_reg_dec += t7 - t6;
      t_reg += t4 - t3;
      t_unreg += t6 - t5;
    }
  }
  reg();
  for (int it = -3; it < calls; ++it) {
    double t0 = now_us();
    enc_dev();
    double t1 = now_us();
    dec_dev();
    double t2 = now_us();
    if (it >= 0) {
      t_res_enc += t1 - t0;
      t_res_dec += t2 - t1;
    }
  }
  check("resident");
  unreg();
  const double cn = calls;
  printf("{\"what\": \"sync RS(10,4) 1 MiB-cell call: staged (hrs_encode/hrs_decode) vs per-call hipHostRegister of "
         "the rows' pages + zero-copy kernels vs pages registered once\", \"calls\": %d, \"same_addr\": %s, "
         "\"staged_encode_us\": %.1f, \"staged_decode_us\": %.1f, \"registered_encode_us\": %.1f, "
         "\"registered_decode_us\": %.1f, \"register_us\": %.1f, \"unregister_us\": %.1f, \"resident_encode_us\": %.1f, "
         "\"resident_decode_us\": %.1f, \"per_row_encode_us\": %.1f, \"per_row_decode_us\": %.1f, "
         "\"registered_pages\": %zu, \"ok\": %s}\n",
         calls, same_addr ? "true" : "false", t_stage_enc / cn, t_stage_dec / cn, t_reg_enc / cn, t_reg_dec / cn,
         t_reg / cn, t_unreg / cn, t_res_enc / cn, t_res_dec / cn, t_rows_enc / cn, t_rows_dec / cn,
         static_cast<size_t>((a1 - a0) / 4096),
         ok ? "true" : "false");
  hrs_destroy(c);
  free(heap);
  return ok ? 0 : 1;
}
