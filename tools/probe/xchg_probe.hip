// tools/probe/xchg_probe.hip -- Table12::xchg/restore (lz4_compress.hip) against a
// sequential model: random chunks of 64 (slot, position, valid) lanes with
// increasing positions, a random match lane ks; after xchg + restore the table
// must equal the sequential loop's (get, put per lane up to ks) and every lane
// <= ks must have read the sequential get.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define KDB_PROBE_ONLY
#include "../../kingdb_amd/csrc/lz4_compress.hip"

using namespace kdb_lz4;

__global__ void run(const uint32_t* slot, const uint32_t* pos, const uint32_t* val, const uint32_t* ks_in,
                    uint32_t trials, uint32_t* refs, uint8_t* tables) {
  __shared__ __attribute__((aligned(16))) uint8_t t[kTable12Bytes];
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = lane; i < kTable12Bytes; i += 64) t[i] = 0;
  __syncthreads();
  Table12 tab(t, t + 8192);
  for (uint32_t c = 0; c < trials; c++) {
    const uint32_t h = slot[c * 64 + lane], p = pos[c * 64 + lane];
    const bool valid = val[c * 64 + lane] != 0;
    const uint32_t r = tab.xchg(h, p, valid);
    refs[c * 64 + lane] = r;
    const uint32_t ks = ks_in[c];
    if (ks < 64) {
      const uint32_t ip = readlane(p, ks);
      if (valid && lane > ks && r <= ip) tab.restore(h, r);
    }
    __syncthreads();
  }
  for (uint32_t i = lane; i < kTable12Bytes; i += 64) tables[i] = t[i];
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 2;   // 0: no match lanes, 1: all valid + no match, 2: full
  const uint32_t trials = 3000;
  std::vector<uint32_t> slot(trials * 64), pos(trials * 64), val(trials * 64), ks(trials);
  srand(11);
  uint32_t p = 1;
  for (uint32_t c = 0; c < trials; c++) {
    const uint32_t K = 1 + rand() % 64;          // slots drawn from a small window: heavy sharing
    const uint32_t base = rand() % (8192 - 64);
    for (int l = 0; l < 64; l++) {
      slot[c * 64 + l] = base + rand() % K;
      pos[c * 64 + l] = (p + l) & 0xfff;
      val[c * 64 + l] = mode == 1 ? 1 : (rand() % 8) != 0;
    }
    ks[c] = (mode == 2 && (rand() % 3)) ? rand() % 64 : 64;       // 64: no match in this chunk
    p += 64;
    if (p > 3900) p = 1;                           // positions must grow within the model's tables
  }
  // the model: sequential get/put, stop after ks
  std::vector<uint32_t> T(8192, 0), expref(trials * 64, 0);
  std::vector<int> chk(trials * 64, 0);
  std::vector<uint32_t> Tcur(8192, 0);
  // positions wrap (p reset) -> a later chunk's positions may be smaller than
  // old entries; the restore rule assumes growth, so reset the model table and
  // the device table only at chunk 0 and keep p monotone within a run segment
  uint32_t *dS, *dP, *dV, *dK, *dR;
  uint8_t* dT;
  hipMalloc(&dS, slot.size() * 4); hipMalloc(&dP, pos.size() * 4); hipMalloc(&dV, val.size() * 4);
  hipMalloc(&dK, ks.size() * 4); hipMalloc(&dR, slot.size() * 4); hipMalloc(&dT, kTable12Bytes);
  // run segments separately so positions grow within each
  long bad_ref = 0, bad_tab = 0, segs = 0;
  uint32_t c0 = 0;
  while (c0 < trials) {
    uint32_t c1 = c0 + 1;
    while (c1 < trials && pos[c1 * 64] > pos[(c1 - 1) * 64]) c1++;
    std::fill(Tcur.begin(), Tcur.end(), 0);
    for (uint32_t c = c0; c < c1; c++) {
      for (uint32_t l = 0; l < 64; l++) {
        if (!val[c * 64 + l]) continue;
        if (ks[c] < 64 && l > ks[c]) break;
        const uint32_t h = slot[c * 64 + l];
        expref[c * 64 + l] = Tcur[h];
        chk[c * 64 + l] = 1;
        Tcur[h] = pos[c * 64 + l];
      }
    }
    const uint32_t n = c1 - c0;
    hipMemcpy(dS, slot.data() + c0 * 64, n * 256, hipMemcpyHostToDevice);
    hipMemcpy(dP, pos.data() + c0 * 64, n * 256, hipMemcpyHostToDevice);
    hipMemcpy(dV, val.data() + c0 * 64, n * 256, hipMemcpyHostToDevice);
    hipMemcpy(dK, ks.data() + c0, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(run, dim3(1), dim3(64), 0, 0, dS, dP, dV, dK, n, dR, dT);
    std::vector<uint32_t> R(n * 64);
    std::vector<uint8_t> TT(kTable12Bytes);
    hipMemcpy(R.data(), dR, n * 256, hipMemcpyDeviceToHost);
    hipMemcpy(TT.data(), dT, kTable12Bytes, hipMemcpyDeviceToHost);
    for (uint32_t i = 0; i < n * 64; i++)
      if (chk[c0 * 64 + i] && R[i] != expref[c0 * 64 + i]) bad_ref++;
    for (uint32_t h = 0; h < 8192; h++) {
      const uint32_t e = TT[h] | (((TT[8192 + (h >> 1)] >> ((h & 1) * 4)) & 15u) << 8);
      if (e != Tcur[h]) bad_tab++;
    }
    segs++;
    c0 = c1;
  }
  printf("mode %d segments %ld: wrong gets %ld, wrong table entries %ld\n", mode, segs, bad_ref, bad_tab);
  return (bad_ref || bad_tab) ? 1 : 0;
}
