/* pcg64.c -- numpy default_rng(seed) restated (TEST INFRASTRUCTURE; see oracle.h).
 *
 * The reference draws cube sizes (scene.py:121-131) and spawn quaternions (task_utils.py:47-52) from
 * np.random.default_rng(seed) = PCG64(SeedSequence(seed)).  Restated from numpy's published
 * algorithm (numpy/random/bit_generator.pyx SeedSequence, numpy/random/src/pcg64): pool of 4 uint32
 * words mixed by hashmix/mix, generate_state(4, uint64) -> 128-bit initstate and initseq,
 * pcg64_srandom_r, XSL-RR 128/64 output; next_double = (next64 >> 11) * 2^-53.
 * Pinned against numpy draws in tests/golden/rng_pcg64.npz.
 */
#include "oracle.h"

typedef unsigned __int128 u128;

#define INIT_A 0x43b0d7e5u
#define MULT_A 0x931e8875u
#define INIT_B 0x8b51f9ddu
#define MULT_B 0x58f38dedu
#define MIX_MULT_L 0xca01f9ddu
#define MIX_MULT_R 0x4973f715u

static uint32_t hashmix(uint32_t value, uint32_t* hc) {
  value ^= *hc;
  *hc *= MULT_A;
  value *= *hc;
  value ^= value >> 16;
  return value;
}

static uint32_t mix(uint32_t x, uint32_t y) {
  uint32_t r = MIX_MULT_L * x - MIX_MULT_R * y;
  r ^= r >> 16;
  return r;
}

static const u128 PCG_MULT = (((u128)0x2360ED051FC65DA4ULL) << 64) | 0x4385DF649FCCF645ULL;

static u128 get_state(const or_pcg64* r) { return ((u128)r->state_hi << 64) | r->state_lo; }
static u128 get_inc(const or_pcg64* r) { return ((u128)r->inc_hi << 64) | r->inc_lo; }
static void put_state(or_pcg64* r, u128 s) {
  r->state_hi = (uint64_t)(s >> 64);
  r->state_lo = (uint64_t)s;
}

void or_pcg64_seed(or_pcg64* r, uint64_t seed) {
  uint32_t ent[2];
  int nent = 0;
  ent[nent++] = (uint32_t)seed;
  if (seed >> 32) ent[nent++] = (uint32_t)(seed >> 32);
  uint32_t pool[4];
  uint32_t hc = INIT_A;
  for (int i = 0; i < 4; i++) pool[i] = hashmix(i < nent ? ent[i] : 0u, &hc);
  for (int s = 0; s < 4; s++)
    for (int d = 0; d < 4; d++)
      if (s != d) pool[d] = mix(pool[d], hashmix(pool[s], &hc));
  uint32_t words[8];
  uint32_t hb = INIT_B;
  for (int i = 0; i < 8; i++) {
    uint32_t v = pool[i % 4];
    v ^= hb;
    hb *= MULT_B;
    v *= hb;
    v ^= v >> 16;
    words[i] = v;
  }
  uint64_t val[4];
  for (int i = 0; i < 4; i++) val[i] = (uint64_t)words[2 * i] | ((uint64_t)words[2 * i + 1] << 32);
  u128 initstate = ((u128)val[0] << 64) | val[1];
  u128 initseq = ((u128)val[2] << 64) | val[3];
  u128 inc = (initseq << 1) | 1;
  r->inc_hi = (uint64_t)(inc >> 64);
  r->inc_lo = (uint64_t)inc;
  u128 st = 0;
  st = st * PCG_MULT + inc;
  st += initstate;
  st = st * PCG_MULT + inc;
  put_state(r, st);
}

uint64_t or_pcg64_next64(or_pcg64* r) {
  u128 st = get_state(r) * PCG_MULT + get_inc(r);
  put_state(r, st);
  uint64_t x = (uint64_t)(st >> 64) ^ (uint64_t)st;
  unsigned rot = (unsigned)(st >> 122);
  return (x >> rot) | (x << ((-rot) & 63));
}

double or_pcg64_double(or_pcg64* r) { return (double)(or_pcg64_next64(r) >> 11) * (1.0 / 9007199254740992.0); }
