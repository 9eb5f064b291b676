// graph_sets.hip — shared-read graph from (read, contig) records (gfx950).
//
// Replaces the pair counting of ReadGraph.from_contigs (karma/read_graph.py:31-49)
// on (read, contig) records (contig.py:24 readsets), DESIGN.md §4.  Output: the
// sorted unique (a << 32 | b, count) list over pairs a <= b of contigs sharing
// reads; the diagonal (a, a) counts |readset(a)|, the weight normaliser.
//
// A read's distinct contigs are "compact" when they lie in [m0, m0 + 3].
// Contigs that share reads are isoforms of one gene, which assemblers list next
// to each other (Trinity: TRINITY_DNx_cy_gz_i1, _i2, ...), so nearly every read
// is compact.  A compact read is one code (m0, M), bit i of (1 | M << 1)
// marking contig m0 + i: dedup and order come for free.  Other reads (wider
// spans) take the general path: sort network, dedup, every pair (p <= q).
//
//   classify    one wave per chunk of 8192 records, no block barriers: lane l
//               walks records 8l..8l+7 of each 512-record step in registers
//               (reads crossing lanes merge by DPP) and writes one u32 code per
//               compact read (ballot-compacted, into the chunk's own region);
//               general reads' starts go to the region's tail, reads of > 8
//               records to the big-read list.
//   general     one wave per chunk with general reads: pairs as u64 keys into
//               the chunk's pair list.
//   partition   (codes, pairs) consecutive chunk lists fill a 64 KB LDS buffer;
//               a full buffer is counting-sorted by bucket in LDS and written
//               as 16-byte-aligned padded runs, one directory row per flush.
//   code reduce per (code bucket, group of flushes): direct-mapped LDS
//               histogram over (m0, M), one no-return LDS add per read.
//   pair reduce per (pair bucket, group of flushes): band counters for
//               b - a < 8 and an LDS hash table for the rest.
//   final       per pair bucket: sums the partials, expands the code histogram
//               into band pairs, merges the hash lists, writes the sorted list.
//   big reads   (> 8 records): separate generic path, merged at the end.
// Device-side counters size every grid-stride loop, so the common path has
// one host synchronisation (flags, overflow, output size) at the end.

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <type_traits>

#include "karma_internal.h"

using namespace karma;

namespace {

#include "graph_device.h"

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kMaxB = 2048;           // pair buckets (n_contigs <= 2^21 keeps the compact path)
constexpr int kMaxBc = 512;           // code buckets
// partition LDS is sized by the bucket count: the narrow variants (<= 512 pair
// and <= 128 code buckets, n_contigs <= 2^19) keep 3 code-partition blocks per CU
constexpr int kNarrowB = 512, kNarrowBc = 128;
#ifndef KARMA_REC_NT
#define KARMA_REC_NT 1  // classify's record loads non-temporal (plain loads: classify 0.53 -> 0.58 ms)
#endif
#ifndef KARMA_PART_LOAD_NT
#define KARMA_PART_LOAD_NT 1  // the partition's loads of classify's codes non-temporal: they are read
                              // once, and the runs it writes stay in the Infinity Cache for the reduce
                              // (partition 0.173 -> 0.169 ms, reduce 0.087 -> 0.084)
#endif
#ifndef KARMA_APPEND_LOAD_NT
#define KARMA_APPEND_LOAD_NT 1  // as KARMA_PART_LOAD_NT, for the append partition (weak-scaled
                                // config 3: 0.277 -> 0.224 ms; its scattered run writes then
                                // combine in the Infinity Cache instead of competing with the codes)
#endif
#ifndef KARMA_RED_LOAD_NT
#define KARMA_RED_LOAD_NT 0  // the reduces' run loads non-temporal (measured 0.087 -> 0.093 ms)
#endif
#ifndef KARMA_CODE_AUX
#define KARMA_CODE_AUX 0  // cache policy of classify's code stores (2, non-temporal: classify
                          // 0.53 -> 0.59 ms, the partition reading them 0.172 -> 0.165)
#endif
#ifndef KARMA_CR_SMAX
#define KARMA_CR_SMAX 64  // code reduce: at most this many pieces per run
#endif
#ifndef KARMA_CR_PIECES
#define KARMA_CR_PIECES 512  // code reduce: split runs into pieces only while a block has < 512 (per-piece cost dominates: 2048 -> 512 took the 8-rank strong reduce 48.6 -> 26.2 us, weak 126 -> 81 us)
#endif
#ifndef KARMA_CR_PIPE
#define KARMA_CR_PIPE 1  // code reduce: barrier-free run stream with the next batch's bounds prefetched (one GPU: 91 -> 75 us)
#endif
#ifndef KARMA_CG_SHIFT
#define KARMA_CG_SHIFT 18  // a code bucket gets one reduce group per 2^18 records it may hold
#endif
#ifndef KARMA_ONE_GROUP_B
#define KARMA_ONE_GROUP_B 128
#endif
#ifndef KARMA_APPEND_MIN_BC
#define KARMA_APPEND_MIN_BC 129  // code_append_kernel from this many code buckets on (n_contigs > 2^19)
#endif
constexpr int kMaxBwCompact = 10;     // compact reads need 2^(bw+3) band counters <= kBand
// the compact path: kMaxB pair buckets of 2^kMaxBwCompact contigs (8 GPUs x 200k
// contigs of a weak-scaled config 3 = 1.6M stay on it)
constexpr int64_t kMaxCompactN = int64_t(kMaxB) << kMaxBwCompact;

struct Geo {
    int bw, bbits, B;  // pair buckets of 2^bw contigs; pair keys a_local << bbits | b
    int bwc, Bc;       // code buckets of 2^bwc contigs (bwc = 0: no compact path)
    int dbits;         // band width 2^dbits (-1: no band)
};

int make_geo(int64_t N, Geo* g) {
    KARMA_CHECK(N >= 1 && N <= (int64_t(1) << 24), KARMA_ERR_ARG, "n_contigs %lld out of range [1, 2^24]",
                (long long)N);
    int bbits = 1;
    while ((int64_t(1) << bbits) < N) ++bbits;
    auto nb = [&](int w) { return (N + (int64_t(1) << w) - 1) >> w; };
    int bw = 4;
#ifndef KARMA_GEO_B
#define KARMA_GEO_B 256  // pair buckets aimed at (A/B builds: more, smaller buckets)
#endif
    while (nb(bw) > KARMA_GEO_B && bw < kMaxBwCompact) ++bw;
    while (nb(bw) > kMaxB) ++bw;
    KARMA_CHECK(bw + bbits <= 31, KARMA_ERR_ARG, "n_contigs too large for 32-bit pair keys");
    g->bw = bw;
    g->bbits = bbits;
    g->B = (int)nb(bw);
    g->dbits = bw + 3 <= 13 ? 3 : (bw <= 13 ? 13 - bw : -1);
    if (bw <= kMaxBwCompact) {
        g->bwc = bw + 2;  // 2^(bwc+3) histogram counters = 128 KB of LDS at most
        g->Bc = (int)nb(g->bwc);
    } else {
        g->bwc = 0;
        g->Bc = 0;
    }
    return KARMA_OK;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Inclusive sum over lanes 0..l of a wave, in DPP steps (row shifts within
// 16-lane rows, then row broadcasts of lanes 15 and 31) instead of ds_bpermute
// round trips through the LDS crossbar.
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return x;
}
// inclusive max over lanes 0..l (values >= -1)
__device__ __forceinline__ int wave_max_incl(int x) {
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xF, 0xF, false));  // row_shr:1
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xF, 0xF, false));  // row_shr:2
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xF, 0xF, false));  // row_shr:4
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xF, 0xF, false));  // row_shr:8
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x142, 0xA, 0xF, false));  // row_bcast:15
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return x;
}
__device__ __forceinline__ uint32_t lane63(uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 63); }


// ---- classify -------------------------------------------------------------------
constexpr int kCW = 256;                // classify threads per block (4 independent waves)
constexpr int kCIter = 512;             // records per wave step (8 per lane; flagged records: 64 x KARMA_FLAG_RPL)
constexpr int kCPer = kCIter / 128;     // 16-byte units per lane per step
#ifndef KARMA_FLAG_RPL
#define KARMA_FLAG_RPL 16  // flagged records per lane and step (16: 1024-record steps, 4 units per lane; 8: 512)
#endif
constexpr uint32_t kContigMask = 0x7FFFFFFFu;  // flagged record: contig id; bit 31 starts a read
constexpr uint32_t kPadW = 0x80000000u;        // flagged padding past a chunk: a read of its own, never emitted
constexpr int64_t kCChunk = 8192;       // records per wave chunk (16 steps; chunk_records may halve it)

struct ClassArgs {
    const uint2* rec;
    int64_t A;
    uint32_t N;
    int compact;
    uint32_t* codes;    // chunk c: [c * chunk, +n_codes[c]) codes, general starts from the end down
    uint32_t* n_codes;  // per chunk
    uint32_t* n_gen;    // per chunk
    unsigned long long* blk_items;  // per partition block (lists_per_block chunks): codes
    int lists_per_block;
    int64_t* big_list;
    unsigned* big_n;
    int* flags;  // 0 order, 1 contig range (2: general pair list full)
    uint32_t* blk_hist;  // per partition block: codes per code bucket (null: no compact path)
    int bwc, Bc;
    const uint32_t* remap;  // contig relabelling (classify2_kernel<.., REMAP>), new id by old id
    int64_t c0;             // first chunk of this launch
    unsigned* skip;         // set: leave the chunks empty (a relabelled rerun follows)
    int64_t chunk;          // records per chunk (chunk_records)
    unsigned* vote = nullptr;  // classify decides the relabel itself (no probe kernel): chunks' votes
    const uint32_t* recw = nullptr;  // FLAG: the records as u32 contig | first-of-read << 31 (RecIn::fw)
};
// In-classify relabel decision (a job without the probe kernel): every
// kVoteStride-th chunk votes when more than 1/8 of its reads are general
// (span > 4 contig ids; the probe's threshold); the kVotes-th vote (half the
// voting chunks' in a small job) sets the relabel word, and chunks that start later skip (their wave reads the word
// as it starts).  The pass is then wasted and reruns relabelled, as after a
// probe; without votes every chunk runs.
constexpr int kVoteStride = 16, kVotes = 4;

// lanes below this one with their bit set in a wave mask
__device__ __forceinline__ int rank_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ---- classify ---------------------------------------------------------------------
// One wave per chunk of 8192 records, no block barriers.  Lane l of a 512-record
// step holds records 8l .. 8l + 7 (coalesced 16-byte loads, transposed through
// the wave's LDS slice) and walks them in order.
//   * a read that starts and ends inside the lane is emitted at its end;
//   * the lane's last read (its "tail") continues into the next lane's
//     "head" (the records before that lane's first read start): the next lane
//     receives the tail (DPP) and emits the merged read; lane 63's tail is
//     carried into the next step's lane 0, and after the chunk's last step
//     into a tail-only pass over the next 8 records;
//   * a read longer than 8 records (a tail plus a head of > 8 records, or a
//     lane without any read start) goes to the big-read list from the lane
//     that merges its tail.
// A read's contigs are tracked as a bit window relative to its first contig
// minus 3: bit (c - fm3), clamped to bit 31 for a contig outside [fm3, fm3 + 30]
// (the read then spans more than 4 contigs).  At the read's end m0 = fm3 +
// ctz(win) and rel = win >> ctz(win): the read is compact when rel < 16 (its
// contigs lie in [m0, m0 + 3]) and m0 < N; it becomes (m0 | M << 24), M =
// rel >> 1.  (m0 < N keeps every bucket and histogram index in range; a
// contig >= N elsewhere in the read is caught by the range check, which fails
// the call.  Testing m0 + 3 < N instead sent the reads of the last gene to the
// general path and woke its whole pipeline: +0.03 ms.)
struct RState {
    uint32_t fm3, win;  // first contig - 3, bits (c - fm3)
};

__device__ __forceinline__ void rs_reset(RState& s, uint32_t c) {
    s.fm3 = c - 3u;
    s.win = 8u;
}
__device__ __forceinline__ void rs_add(RState& s, uint32_t c) { s.win |= 1u << min(c - s.fm3, 31u); }
// compact code of a read: *code valid when the result is true
template <bool COMPACT>
__device__ __forceinline__ bool rs_code(const RState& s, uint32_t N, uint32_t* code) {
    const uint32_t z = (uint32_t)__builtin_ctz(s.win);  // bit 3 (the first contig) is always set
    const uint32_t rel = s.win >> z, m0 = s.fm3 + z;
    *code = m0 | (rel >> 1) << 24;
    return COMPACT && rel < 16u && m0 < N;
}
// the same for a read seen in two parts (a tail and the next lane's head).  A
// marker bit shifted out of 32 bits leaves the first contig's bit at >= 4, so
// the read is still general.
template <bool COMPACT>
__device__ __forceinline__ bool rs_code2(const RState& a, const RState& b, uint32_t N, uint32_t* code) {
    const uint32_t za = (uint32_t)__builtin_ctz(a.win), zb = (uint32_t)__builtin_ctz(b.win);
    const uint32_t ma = a.fm3 + za, mb = b.fm3 + zb, m0 = min(ma, mb);
    const uint32_t rel = ((a.win >> za) << min(ma - m0, 31u)) | ((b.win >> zb) << min(mb - m0, 31u));
    *code = m0 | (rel >> 1) << 24;
    return COMPACT && rel < 16u && m0 < N;
}

// lane-mask forms for the wave's walk: the compares go straight into SGPR lane
// masks, which feed selects through inverse ballots (no 0/1 VGPR round trips)
__device__ __forceinline__ uint64_t lanes(bool c) { return __builtin_amdgcn_ballot_w64(c); }
__device__ __forceinline__ bool in_mask(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
// K23 (the binned classify's staged codes): m0 << 4 | rel, one shift-or
// (rel < 16 on the compact path, bit 0 always set), so that the bucket queue's
// u16 value (m0_local << 3 | M) is one bit-field extract and the bucket one
// shift.  K23 also drops the m0 < N test: m0 >= N needs a contig >= N, which the
// range check reports (the call fails), and bin_emit clamps the bucket so that
// such a code stays inside the queues meanwhile (one op per staged code instead
// of one compare per record)
// (*m0_out: the read's first contig at full width -- K23's m0 << 4 drops its
// top 4 bits -- for the replay's exact range check)
template <bool COMPACT, bool K23 = false>
__device__ __forceinline__ uint64_t rs_code_m(const RState& s, uint32_t N, uint32_t* code, uint32_t* m0_out) {
    const uint32_t z = (uint32_t)__builtin_ctz(s.win);
    const uint32_t rel = s.win >> z, m0 = s.fm3 + z;
    *code = K23 ? m0 << 4 | rel : m0 | (rel >> 1) << 24;
    *m0_out = m0;
    return COMPACT ? lanes(rel < 16u) & (K23 ? ~0ull : lanes(m0 < N)) : 0ull;
}
template <bool COMPACT, bool K23 = false>
__device__ __forceinline__ uint64_t rs_code2_m(const RState& a, const RState& b, uint32_t N, uint32_t* code,
                                               uint32_t* m0_out) {
    const uint32_t za = (uint32_t)__builtin_ctz(a.win), zb = (uint32_t)__builtin_ctz(b.win);
    const uint32_t ma = a.fm3 + za, mb = b.fm3 + zb, m0 = min(ma, mb);
    const uint32_t rel = ((a.win >> za) << min(ma - m0, 31u)) | ((b.win >> zb) << min(mb - m0, 31u));
    *code = K23 ? m0 << 4 | rel : m0 | (rel >> 1) << 24;
    *m0_out = m0;
    return COMPACT ? lanes(rel < 16u) & (K23 ? ~0ull : lanes(m0 < N)) : 0ull;
}

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t old, uint32_t v) {  // lane l <- lane l - 1; lane 0 <- old
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

#ifndef KARMA_CLS_DEFER_RARE
#define KARMA_CLS_DEFER_RARE 1  // general / big reads of a step emitted by a replay after the chunk's loop
                                // (the second walk inside the loop spilled 158 SGPRs: 222M -> 183M VALU)
#endif
constexpr int kRareMax = int(kCChunk / kCIter);  // steps per chunk
constexpr int kRareW = 5;                        // words per listed step
#ifndef KARMA_CLS_RANGE_CODE
#define KARMA_CLS_RANGE_CODE 3  // binned flagged classify: 1 the walk on raw words, 2 the range checked per code (RC)
#endif
#ifndef KARMA_CLS_PACKED
#define KARMA_CLS_PACKED 0  // binned flagged walk: own reads staged as (fm3 << 8 | 8-bit window), coded in bin_stage
#endif
#ifndef KARMA_CLS_EMIT_DUMMY
#define KARMA_CLS_EMIT_DUMMY 0  // binned flagged walk: every lane stores its code (no exec-mask branch per record)
#endif
#ifndef KARMA_CLS_HLEN_MAIN
#define KARMA_CLS_HLEN_MAIN 0  // 1: the main pass tracks the head's length per record too (the round-6 walk)
#endif
#ifndef KARMA_CLS_PIN
#define KARMA_CLS_PIN 2  // walk state pinned per record (see the walk): 1 with 16 records per lane, 2 always
#endif
#ifndef KARMA_CLS_NO_RARE
#define KARMA_CLS_NO_RARE 0  // measurement only (A/B of the rare pass's register cost): no general / big reads emitted
#endif
#ifndef KARMA_CLS2_WAVES
#define KARMA_CLS2_WAVES 4  // 4: 0.541 ms; 5 (84 VGPRs): 0.545; 6 (80 VGPRs, 7 spilled): 0.576
#endif

// ---- binned classify (BIN): compact codes straight into bucket runs --------------
// With few code buckets (Bc <= kBinMaxBc: n_contigs <= 229,376 at bwc = 12)
// each wave keeps one LDS queue of kBinQ u16 codes (m0_local << 3 | M) per
// code bucket.  A code goes to its bucket's queue (one returning LDS add for
// its slot, one 2-byte LDS store); a queue that fills is written out as one
// 128-byte segment (8 lanes x 16 B) at the BACK of the chunk's segment region,
// its bucket id in the chunk's directory; at the chunk's end every non-empty
// queue is written at the FRONT, in bucket order, as a run of 16-byte
// granules (its last one padded with 0xFFFF).  The chunk's header holds each
// bucket's front granule count (a nibble: bucket b's run starts at the sum of
// the nibbles below b), the back count, the back mask and the first 16
// directory bytes.  The code reduce then reads each bucket's runs directly:
// the u32 code stream, the partition kernel and its u16 runs (1.2 GB of
// intermediate traffic at config 3) are gone.
constexpr int kBinQ = 64;        // codes per queue and per back segment (128 B)
constexpr int kBinMaxBc = 56;    // code buckets with a queue (LDS: 56 x 128 B per wave; 7 nibble words)
// header (4 x uint4 per chunk): x0..x6 granule nibbles of buckets 0..55, x7
// back count, x8-x9 back mask, x10-x13 directory bytes 0..15, x14 codes
constexpr int kBinHdr = 4;
struct BinArgs {
    uint16_t* segs;     // per chunk: seg_cap x kBinQ codes (front runs, then back segments from the end)
    uint4* hdr;         // per chunk: kBinHdr uint4 (above)
    uint8_t* dir;       // per chunk: dir_cap bucket ids of the back segments (in flush order)
    int64_t seg_cap;    // segments per chunk: chunk / kBinQ + Bc
    int dir_cap;        // chunk / kBinQ
    int slotted;        // front runs as whole 128-byte slots, slot b = bucket b (see classify2_kernel's end)
};

// HIST: per-block code-bucket histograms for code_append_kernel; COMPACT: the
// compact-code path exists (n_contigs <= 2^21); REMAP: contig ids relabelled
// through P.remap as they are read (contig order without locality, see
// relabel); BIN: codes into bucket segments (see above; not with HIST)
// FLAG: flagged records (4 bytes each, read starts flagged; RecIn): a
// 512-record step is 2 KB (two 16-byte units per lane), no read ids to
// compare or order-check
template <bool HIST, bool COMPACT, bool REMAP = false, bool BIN = false, bool FLAG = false>
__global__ void __launch_bounds__(kCW) __attribute__((amdgpu_waves_per_eu(KARMA_CLS2_WAVES, KARMA_CLS2_WAVES)))
classify2_kernel(ClassArgs P, BinArgs Q) {
    static_assert(!(HIST && BIN), "the binned classify has no partition block histograms");
    // P's fields only the rare steps' replay uses (after the chunk's loop),
    // read there from the kernel argument segment behind an opaque pointer: so
    // they are not held in SGPRs across the hot loop (r05 measured the same
    // re-read INSIDE the loop 0.036 ms slower; here no load is in the loop)
    auto PA = [&]() -> const ClassArgs& {
        if (!KARMA_CLS_DEFER_RARE) return P;
        const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ka));
        return *reinterpret_cast<const ClassArgs*>(ka);
    };
    // records per lane and per step: flagged steps hold twice as many records
    // in the same 16 bytes per lane and unit (the per-step work -- the merge
    // of tails and heads, the transposes' waits, the carry -- then amortises
    // over 1024 records)
    constexpr int RPL = FLAG ? KARMA_FLAG_RPL : 8;
    constexpr int64_t kIt = 64 * RPL;
    constexpr int kFPer = RPL / 4;  // FLAG: 16-byte units per lane and step
    static_assert(RPL == 8 || (FLAG && RPL == 16), "8 or 16 records per lane (16: flagged only)");
    static_assert(!FLAG || kFPer <= kCPer, "the step's units fit the register set");
    // RC: the binned flagged walk reads the raw words (no per-record mask of the
    // start flag) and checks the contig range per code instead of per record:
    // a staged compact code with m0 >= N - 3 (its contigs are m0 .. m0 + 3 at
    // most) lists its step for the replay, which checks the step's compact codes
    // exactly; general and big reads are checked where their records are read
    // (general_kernel, big_pairs_kernel); the chunk-end tail read here
    constexpr bool RC = BIN && FLAG && (KARMA_CLS_RANGE_CODE & 2) && KARMA_CLS_DEFER_RARE;
    constexpr bool RAW = FLAG && (KARMA_CLS_RANGE_CODE & 1);  // the walk on raw words (measurement split)
    // PK: the binned flagged walk stages each own read's state as it ends,
    // (fm3 << 8 | win) with an 8-bit window (bit 7: a contig outside [fm3,
    // fm3 + 6]), one shift-or per record; bin_stage turns 64 of them at a time
    // into codes and lists the step when one is not compact.  fm3 keeps 24
    // bits there, so the range guard lists steps with any contig >= 2^24
    constexpr bool PK = RC && RAW && RPL > 8 && KARMA_CLS_PACKED;
    constexpr uint32_t kWinTop = PK ? 7u : 31u;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t chunk = P.c0 + (int64_t)blockIdx.x * (kCW / 64) + wave;
    const int64_t c_lo = chunk * P.chunk;
    if (c_lo >= P.A) return;  // waves are independent (wave-private LDS only)
    const int64_t c_hi = min(P.A, c_lo + P.chunk);
    uint32_t* out = P.codes + c_lo;
    // the chunk's region as a buffer resource built from wave-uniform values
    const uint64_t out_u = (uint64_t)out;
    const __amdgpu_buffer_rsrc_t out_rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(out_u >> 32)) << 32) |
                                (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)out_u)),
        0, (int)(P.chunk * 4), 0x00020000);
    // transpose buffer: lane l's 8 records in row l (4 units of 16 bytes), the
    // unit index XOR-ed with (l >> 2) & 3: conflict-free for the 16-byte stores
    // (8-lane groups, banks mod 32) and for the row reads (16-lane groups,
    // banks mod 64) alike.  BIN: half of it (rows of lanes 0-31, then of lanes
    // 32-63), to leave LDS for the bucket queues at 4 blocks per CU.
    constexpr int kRows = BIN ? 32 : 64;
    // (+ 16 granules: the emit's slots for lanes without a code, KARMA_CLS_EMIT_DUMMY)
    constexpr int kDummy = BIN && FLAG && KARMA_CLS_EMIT_DUMMY ? 16 : 0;
    __shared__ __attribute__((aligned(16))) u32x4 tbuf[kCW / 64][kRows * 4 + kDummy];
    u32x4* tb = tbuf[wave];
    // the chunk's codes per code bucket, added to its partition block's row at the end
    __shared__ uint32_t whist[kCW / 64][HIST ? kMaxBc : 1];
    uint32_t* wh = whist[wave];
    // BIN: the bucket queues, their fill counts, and rank -> bucket of the end flush
    __shared__ __attribute__((aligned(16))) uint16_t bq[kCW / 64][BIN ? kBinMaxBc * kBinQ : 8];
    __shared__ uint32_t bcnt[kCW / 64][BIN ? kBinMaxBc : 1];
    uint16_t* const q = bq[wave];
    uint32_t* const qn = bcnt[wave];
    // back-segment bookkeeping, touched only when a queue fills (kept in LDS,
    // not in registers across the walk): [0] back count, [1..2] back mask,
    // [3..6] the first 16 directory bytes (for the header)
    __shared__ uint32_t bback[kCW / 64][BIN ? 8 : 1];
    uint32_t* const bst = bback[wave];
    // steps with a general or big read, replayed after the chunk's main loop
    // (kRareW words each: step index | carry flags, the carried tail's state,
    // the previous record's read id), so the hot loop holds no second walk
    __shared__ uint32_t rlist[kCW / 64][KARMA_CLS_DEFER_RARE ? kRareMax * kRareW : 1];
    uint32_t* const rl = rlist[wave];
    uint32_t n_rare = 0;  // uniform
    constexpr bool hist_on = HIST;
    if (hist_on) {
        for (int b = lane; b < P.Bc; b += 64) wh[b] = 0;
        wave_sync();
    }
    if (BIN) {
        if (lane < P.Bc) qn[lane] = 0;
        if (lane < 8) bst[lane] = 0;
        wave_sync();
    }
    // BIN: codes of the lanes in `m` into their queues; a queue that fills is
    // written as a back segment, and the codes that found it full go into the
    // emptied queue (a queue holds < kBinQ codes between calls, so the lane
    // that took slot kBinQ - 1 exists whenever one overflowed)
    // (code: the K23 form m0 << 4 | rel, rel's bit 0 set: bits 1.. are
    // m0_local << 3 | M, bits bwc + 4.. the bucket)
    auto bin_emit = [&](uint64_t m, uint32_t code) {
        const uint32_t bk = min(code >> (P.bwc + 4), (uint32_t)P.Bc - 1u);
        const uint16_t val = (uint16_t)__builtin_amdgcn_ubfe(code, 1u, (uint32_t)P.bwc + 3u);
        uint32_t pos = 0;
        if (in_mask(m)) {
            pos = __hip_atomic_fetch_add(&qn[bk], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (pos < (uint32_t)kBinQ) {
                uint32_t qi = (bk << 6) + pos;
                asm("" : "+v"(qi));  // two shift-adds, not two shifts and an add
                q[qi] = val;
            }
        }
        uint64_t full = m & lanes(pos == (uint32_t)kBinQ - 1u);
        if (!full) return;
        const uint64_t over = m & lanes(pos >= (uint32_t)kBinQ);
        while (full) {  // rare: ~1 per kBinQ codes of a bucket (uniform loop)
            const int L = __builtin_ctzll(full);
            full &= full - 1;
            const uint32_t fb = (uint32_t)__builtin_amdgcn_readlane((int)bk, L);
            wave_lds_order();
            const uint32_t nbk = (uint32_t)__builtin_amdgcn_readfirstlane((int)bst[0]);
            const BinArgs& Qa = Q;
            uint16_t* const dst = Qa.segs + (chunk * Qa.seg_cap + Qa.seg_cap - 1 - (int64_t)nbk) * kBinQ;
            if (lane < 8) {
                const u32x4 v = *reinterpret_cast<const u32x4*>(q + fb * kBinQ + 8 * lane);
                *reinterpret_cast<u32x4*>(dst + 8 * lane) = v;
            }
            if (lane == 0) {
                Qa.dir[chunk * Qa.dir_cap + nbk] = (uint8_t)fb;
                bst[0] = nbk + 1;
                bst[1 + (fb >> 5)] |= 1u << (fb & 31);
                if (nbk < 16) bst[3 + (nbk >> 2)] |= fb << (8 * (nbk & 3));
            }
            wave_lds_order();
            if (in_mask(over) && bk == fb) q[fb * kBinQ + pos - kBinQ] = val;
            if (lane == 0) qn[fb] -= (uint32_t)kBinQ;  // was kBinQ + the overflowed codes
            wave_lds_order();
        }
    };
    // BIN: a step's codes are staged (ballot-compacted u32) in the transpose
    // buffer, idle during the walk (a step ends <= 512 reads: 2 KB), and go
    // into the queues once per step, 64 at a time, instead of at each of the
    // walk's 8 emit points
    uint32_t* const stg = reinterpret_cast<uint32_t*>(tb);
    const uint32_t* const stg_l = stg + lane;
    uint32_t* const stg_dummy = stg + 16 * kRows + lane;  // (kDummy)
    uint32_t ns = 0;  // staged codes (uniform)
    uint32_t nc = 0, ng = 0;  // the chunk's codes and general reads
    // one value per lane of `b` into the staging area (kDummy: every lane
    // stores, the others into a slot of their own past it: no exec-mask branch)
    auto stage = [&](uint64_t b, uint32_t v) {
        if (kDummy) {
            uint32_t r = (uint32_t)rank_below(b);
            asm volatile("" : "+v"(r));  // in every lane, then one select of the address
            uint32_t* const sp = in_mask(b) ? stg + ns + r : stg_dummy;
            *sp = v;
        } else if (in_mask(b)) {
            stg[ns + (uint32_t)rank_below(b)] = v;
        }
        ns += __popcll(b);
    };
    static_assert(kBinQ == 64, "queue slots: bk << 6");
    // RC: staged codes whose contigs may reach N (m0 >= N - 3), this step
    uint64_t stage_hi = 0, hi_next = 0;
    const uint32_t code_hi = ((uint32_t)max(P.N, 3u) - 3u) << 4;
    auto bin_stage = [&]() {
        if (!ns) return;
        wave_lds_order();
        for (uint32_t j0 = 0; j0 < ns; j0 += 64) {
            // unpredicated read (ns <= 512 codes: the 2 KB buffer; j0 + lane < 512 always; past ns masked off)
            uint32_t cd = stg_l[j0];
            uint64_t m = lanes((uint32_t)lane < ns - j0);
            if (PK) {
                // (fm3 << 8 | win) -> m0 << 4 | rel: q = m0 << 8 | win (mod 2^32)
                const uint32_t win = cd & 255u, z = (uint32_t)__builtin_ctz(win), rel = win >> z;
                const uint32_t q = cd + (z << 8);
                cd = ((q >> 4) & ~15u) | rel;
                const uint64_t okm = m & lanes(rel < 16u);
                stage_hi |= m & ~okm;  // a general or big read: the step goes to the replay
                m = okm;
                nc += __popcll(okm);
            }
            if (RC) stage_hi |= m & lanes(cd >= code_hi);
            bin_emit(m, cd);
        }
        ns = 0;
        wave_lds_order();
    };

    // records [t0, hi) of a step, coalesced: unit u of lane l = records t0 + 128u + 2l, + 1.
    // Past the chunk: read id kEmpty (a read of its own that is never emitted), contig 0.
    auto prefetch = [&](u32x4 (&dst)[kCPer], int64_t t0, int64_t hi) {
        if (FLAG) {  // unit u of lane l = records t0 + 256u + 4l .. + 3; past the chunk: a read start, contig 0
            const int64_t gw = t0 + 4 * lane;
            if (t0 + kIt <= hi) {
#pragma unroll
                for (int u = 0; u < kFPer; ++u)
                    dst[u] = KARMA_REC_NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(P.recw + gw + 256 * u))
                                          : *reinterpret_cast<const u32x4*>(P.recw + gw + 256 * u);
            } else {
#pragma unroll
                for (int u = 0; u < kFPer; ++u) {
                    const int64_t gi = gw + 256 * u;
                    dst[u] = u32x4{gi < hi ? P.recw[gi] : kPadW, gi + 1 < hi ? P.recw[gi + 1] : kPadW,
                                   gi + 2 < hi ? P.recw[gi + 2] : kPadW, gi + 3 < hi ? P.recw[gi + 3] : kPadW};
                }
            }
            return;
        }
        const int64_t gb = t0 + 2 * lane;
        if (t0 + kIt <= hi) {
#pragma unroll
            for (int u = 0; u < kCPer; ++u)
                if (KARMA_REC_NT)
                    dst[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(P.rec + gb + 128 * u));
                else
                    dst[u] = *reinterpret_cast<const u32x4*>(P.rec + gb + 128 * u);
        } else {
#pragma unroll
            for (int u = 0; u < kCPer; ++u) {
                const int64_t gi = gb + 128 * u;
                const uint2 r0 = gi < hi ? P.rec[gi] : make_uint2(kEmpty, 0u);
                const uint2 r1 = gi + 1 < hi ? P.rec[gi + 1] : make_uint2(kEmpty, 0u);
                dst[u] = u32x4{r0.x, r0.y, r1.x, r1.y};
            }
        }
    };
    // carry from the previous lane 63: its last read id, and its tail read
    bool have_prev = c_lo > 0;
    uint32_t prev_rid = FLAG || !have_prev ? kEmpty : P.rec[c_lo - 1].x;
    bool ct_ok = false;  // a tail read (started in this chunk) is carried
    RState ct{};
    uint32_t ct_len = 0, ct_pos = 0;
    uint64_t bad_order = 0, bad_contig = 0;  // lane masks
    // one 512-record step from `buf`, which then takes the next step's loads
    // (two steps in flight -- a second register set at 4 waves/SIMD -- measured
    // the same: the walk already runs at ~5.7 TB/s of records + codes)
    // FULL: all 512 records of the step are inside the chunk (every step but a
    // chunk's last): no per-record validity tests
    // REMAP: the contigs of the step after next are relabelled here (gathers
    // from the remap table into `nxt`, loaded a step earlier), a full step
    // before they are used; `buf` then takes the records two steps ahead
    auto remap_units = [&](u32x4 (&b)[kCPer]) {
        if (FLAG) {  // the low 31 bits relabelled, the read-start flag kept
            auto rm = [&](uint32_t w) {
                const uint32_t c = w & kContigMask;
                return c < P.N ? P.remap[c] | (w & ~kContigMask) : w;
            };
#pragma unroll
            for (int u = 0; u < kFPer; ++u) b[u] = u32x4{rm(b[u].x), rm(b[u].y), rm(b[u].z), rm(b[u].w)};
            return;
        }
#pragma unroll
        for (int u = 0; u < kCPer; ++u) {  // ids out of range stay out of range (the range check fails the call)
            b[u].y = b[u].y < P.N ? P.remap[b[u].y] : b[u].y;
            b[u].w = b[u].w < P.N ? P.remap[b[u].w] : b[u].w;
        }
    };
    // REPLAY: a rare step again, after the main loop: its records reloaded and
    // its carry-in restored; only the general / big reads are emitted
    auto step = [&](auto full_tag, auto replay_tag, u32x4 (&buf)[kCPer], u32x4 (&nxt)[kCPer], int64_t t0) {
        constexpr bool FULL = decltype(full_tag)::value;
        constexpr bool REPLAY = decltype(replay_tag)::value;
        uint32_t rid[RPL], ctg[RPL];  // FLAG: rid holds the raw words (bit 31: a read starts here)
        // loader lane L, unit u -> lane 16u + L/4, unit L & 3; lane l reads its 8 records back
        if constexpr (FLAG && RPL == 16) {
            // two passes of 128 granules (2 KB: BIN's half buffer): pass h holds
            // units 2h, 2h + 1 = the records of lanes 32h .. 32h + 31; local
            // granule g at slot g ^ ((g >> 4) & 3): the stores' 8-lane groups
            // stay in one 16-granule row (a permutation of it), and the reads'
            // 16-lane groups (granules 4j + k) fall on 16 distinct bank quads
            const int rl = lane & 31;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int g = 64 * u + lane;
                    tb[g ^ ((g >> 4) & 3)] = buf[2 * h + u];
                }
                wave_sync();
                if ((lane >> 5) == h) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int g = 4 * rl + k;
                        const u32x4 qv = tb[g ^ ((g >> 4) & 3)];
                        rid[4 * k] = qv.x, rid[4 * k + 1] = qv.y, rid[4 * k + 2] = qv.z, rid[4 * k + 3] = qv.w;
                    }
                }
                wave_sync();
            }
#pragma unroll
            for (int i = 0; i < RPL; ++i) ctg[i] = rid[i] & kContigMask;
        } else if (FLAG) {
            // 16-byte granule g = 64u + L (records 4g .. 4g + 3) at slot g ^ ((g >> 3) & 1): lane l
            // reads granules 2l, 2l + 1 (conflict-free on both sides; 2 KB: BIN's half buffer)
#pragma unroll
            for (int u = 0; u < kFPer; ++u) {
                const int g = 64 * u + lane;
                tb[g ^ ((g >> 3) & 1)] = buf[u];
            }
            wave_sync();
            const int sw = (lane >> 2) & 1;
            const u32x4 q0 = tb[(2 * lane) ^ sw], q1 = tb[(2 * lane + 1) ^ sw];
            rid[0] = q0.x, rid[1] = q0.y, rid[2] = q0.z, rid[3] = q0.w;
            rid[4] = q1.x, rid[5] = q1.y, rid[6] = q1.z, rid[7] = q1.w;
            wave_sync();
#pragma unroll
            for (int i = 0; i < 8; ++i) ctg[i] = rid[i] & kContigMask;
        } else if (!BIN) {
#pragma unroll
            for (int u = 0; u < kCPer; ++u) {
                const int row = 16 * u + (lane >> 2);
                tb[4 * row + ((lane & 3) ^ ((row >> 2) & 3))] = buf[u];
            }
            wave_sync();
#pragma unroll
            for (int u = 0; u < kCPer; ++u) {
                const u32x4 qv = tb[4 * lane + (u ^ ((lane >> 2) & 3))];
                rid[2 * u] = qv.x;
                ctg[2 * u] = qv.y;
                rid[2 * u + 1] = qv.z;
                ctg[2 * u + 1] = qv.w;
            }
            wave_sync();
        } else {
            // two halves through 32 rows: units 0-1 hold lanes 0-31's records,
            // units 2-3 lanes 32-63's; every lane reads row (lane & 31) in both
            // halves and keeps the one of its own
            const int rl = lane & 31;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int row = 16 * u + (lane >> 2);
                    tb[4 * row + ((lane & 3) ^ ((row >> 2) & 3))] = buf[2 * h + u];
                }
                wave_sync();
                if ((lane >> 5) == h) {
#pragma unroll
                    for (int u = 0; u < kCPer; ++u) {
                        const u32x4 qv = tb[4 * rl + (u ^ ((rl >> 2) & 3))];
                        rid[2 * u] = qv.x;
                        ctg[2 * u] = qv.y;
                        rid[2 * u + 1] = qv.z;
                        ctg[2 * u + 1] = qv.w;
                    }
                }
                wave_sync();
            }
        }
        if (REPLAY) {
        } else if (REMAP) {
            if (t0 + kIt < c_hi) remap_units(nxt);
            if (t0 + 2 * kIt < c_hi) prefetch(buf, t0 + 2 * kIt, c_hi);
        } else if (t0 + kIt < c_hi) {
            prefetch(buf, t0 + kIt, c_hi);
        }
        // valid records of this lane (own reads start at a valid record)
        const int nval = FULL ? RPL : (int)max<int64_t>(0, min<int64_t>(RPL, c_hi - (t0 + RPL * lane)));
        const uint32_t prev_last = FLAG ? 0u : dpp_shr1(prev_rid, rid[RPL - 1]);
        // order and range checks as lane masks (padding: read id kEmpty, contig
        // 0); the order of records inside the lane is checked during the walk
        if (!REPLAY) {
            if (!FLAG) bad_order |= lanes(prev_last > rid[0]) & (have_prev ? ~0ull : ~1ull);
            if (!RC) {
                uint32_t cmax = ctg[0];
#pragma unroll
                for (int i = 1; i < RPL; ++i) cmax = max(cmax, ctg[i]);
                bad_contig |= lanes(cmax >= P.N);
            } else {
                // a contig >= 2^28 would wrap out of the staged code's m0 << 4
                // (and pass the per-code test below): its step goes to the
                // replay, which checks at full width (one OR per record)
                // (and the next step too when lane 63 holds one: its tail read
                // is emitted there)
                uint32_t o = rid[0];
#pragma unroll
                for (int i = 1; i < RPL; ++i) o |= rid[i];
                const uint64_t hi = lanes((o & (PK ? 0x7F000000u : 0x70000000u)) != 0u);
                stage_hi |= hi | hi_next;
                hi_next = hi >> 63;
            }
        }
        const uint32_t ubase = (uint32_t)(t0 - c_lo) + (uint32_t)RPL * lane;
        // The lane's walk (branch-free: no lane predicate lives across a branch,
        // so the compiler keeps them as SGPR lane masks).  Emission: codes from
        // the front of the chunk's region (BIN: into the bucket queues),
        // general read starts (chunk-relative) from the back, big reads to the
        // big list.  The walk runs once for the codes; only when some lane met
        // a general or a big read does it run again to emit those (rare on
        // assembled transcriptomes).  Codes go out through a buffer store whose
        // range check drops the lanes without one.
        // Outputs: the lane's last read (st, spos), whether one started in the
        // lane, and the mask of lanes with a general or big read.
        auto walk = [&](auto rare_pass, RState& st, uint32_t& spos, uint64_t& started) -> uint64_t {
            constexpr bool RARE = decltype(rare_pass)::value;
            uint64_t rare = 0;
            // e: lanes where a read ends here; ok: ... it is compact (code); big: ... it has > 8 records
            auto emit = [&](uint64_t e, uint64_t ok, uint32_t code, uint32_t m0, uint32_t pos, uint64_t big) {
                if (!RARE) {
                    const uint64_t b = e & ok & ~big;
                    if (PK) {  // (the merged read; counted in bin_stage) m0 - 3, rel at bit 3
                        stage(b, (m0 - 3u) << 8 | (code & 15u) << 3);
                        rare |= e & (big | ~ok);
                        return;
                    }
                    if (BIN) {
                        stage(b, code);
                    } else {
                        // lanes without a code store past the region (bit 31): dropped
                        const uint32_t boff =
                            ((nc + (uint32_t)rank_below(b)) * 4u) | (in_mask(b) ? 0u : 0x80000000u);
                        __builtin_amdgcn_raw_buffer_store_b32(code, out_rsrc, (int)boff, 0, KARMA_CODE_AUX);
                    }
                    if (hist_on && in_mask(b)) atomicAdd(&wh[(code & 0xFFFFFFu) >> P.bwc], 1u);
                    nc += __popcll(b);
                    rare |= e & (big | ~ok);
                } else {
                    if (RC) {  // the step's compact codes (m0 << 4 | rel): their top contig < N
                        const uint64_t cm = e & ok & ~big;
                        if (cm)
                            bad_contig |= cm & lanes(m0 + 31u - (uint32_t)__builtin_clz(code & 15u) >= PA().N);
                    }
                    const uint64_t g = e & ~big & ~ok;
                    if (g) {
                        const ClassArgs& Pa = PA();
                        if (in_mask(g)) (Pa.codes + c_lo)[Pa.chunk - 1 - (ng + rank_below(g))] = pos;
                        ng += __popcll(g);
                    }
                    const uint64_t bg = e & big;
                    if (bg) {
                        if (in_mask(bg)) {
                            const ClassArgs& Pa = PA();
                            Pa.big_list[atomicAdd(Pa.big_n, 1u)] = c_lo + pos;
                        }
                    }
                }
            };
            // S(i): lanes where a read starts at record i (lane 0 of a chunk's
            // first step: always); computed where used, so few masks are live
            auto S = [&](int i) -> uint64_t {
                if (FLAG) return lanes((int)rid[i] < 0) | (i == 0 && !have_prev ? 1ull : 0ull);
                return i == 0 ? lanes(rid[0] != prev_last) | (have_prev ? 0ull : 1ull) : lanes(rid[i] != rid[i - 1]);
            };
            const uint64_t S0 = S(0);
            RState hd;
            rs_reset(st, ctg[0]);
            hd = st;
            spos = 0;
            uint32_t hlen = in_mask(S0) ? 0u : (uint32_t)RPL;  // head: records before the first start (RPL: none)
            // the head's length matters only for a non-compact read (general or
            // big), whose step the main pass lists for the replay anyway: with
            // 16 records per lane the main pass needs only "no start in the
            // lane" (~started), one select per record less
            constexpr bool HLEN = RARE || RPL <= 8 || KARMA_CLS_HLEN_MAIN;
            started = S0;
            uint64_t Si = S0;
#pragma unroll
            for (int i = 0; i < RPL; ++i) {
                // 16 records per lane: <= 64 codes per emit point, 16 of them --
                // the first eight's codes go into the queues mid-walk (the staging
                // buffer holds 512)
                if (!RARE && BIN && RPL > 8 && i == 8) bin_stage();
                if (i > 0) {
                    const uint64_t cap = Si & ~started;  // the first start: the head ends here
                    hd.win = in_mask(cap) ? st.win : hd.win;
                    if (HLEN) hlen = in_mask(cap) ? (uint32_t)i : hlen;
                    started |= Si;
                    spos = in_mask(Si) ? (uint32_t)i : spos;
                    if (RAW) {
                        // raw word: bit 31 set exactly at a start (i > 0), so a
                        // start's contig - 3 is w - 0x80000003, and another
                        // record's w is its contig
                        const uint32_t w = rid[i];
                        const uint32_t fm3 = in_mask(Si) ? w - 0x80000003u : st.fm3;
                        st.win = in_mask(Si) ? 8u : st.win | (1u << min(w - fm3, kWinTop));
                        st.fm3 = fm3;
                    } else {
                        const uint32_t c = ctg[i];
                        const uint32_t fm3 = in_mask(Si) ? c - 3u : st.fm3;
                        // a new read: bit 3 alone (c - fm3 = 3)
                        st.win = (in_mask(Si) ? 0u : st.win) | (1u << min(c - fm3, 31u));
                        st.fm3 = fm3;
                    }
                    if (!RARE && !FLAG) bad_order |= lanes(rid[i - 1] > rid[i]);
                }
                if (i < RPL - 1) {
                    // an own read ends at i (the next record starts one); it
                    // started at a valid record iff i < nval
                    const uint64_t Sn = S(i + 1);
                    const uint64_t e = Sn & started & (FULL ? ~0ull : lanes(i < nval));
                    Si = Sn;
                    if (PK && !RARE) {  // the read's state, coded in bin_stage
                        stage(e, st.fm3 << 8 | st.win);
                    } else {
                        uint32_t code, m0;
                        const uint64_t ok = rs_code_m<COMPACT, BIN>(st, P.N, &code, &m0);
                        // an own read of > 8 records (16 per lane) that is not
                        // compact is a big read (the general path reads 8); a compact
                        // one is a code like any other (its contig set is the code)
                        const uint64_t big_own =
                            RARE && i + 1 > kMaxFast ? lanes((uint32_t)i + 1u - spos > (uint32_t)kMaxFast) & ~ok : 0ull;
                        emit(e, ok, code, m0, ubase + spos, big_own);
                    }
                }
                // 16 records: pin the walk's state at each record, or the compiler
                // sinks the head's selects and the rare mask past the loop and
                // keeps every record's lane masks alive for them (SGPRs spilled
                // into VGPR lanes)
                if (KARMA_CLS_PIN > 1 || (RPL > 8 && KARMA_CLS_PIN)) {
                    asm volatile("" : "+v"(hd.win), "+v"(spos), "+v"(st.win), "+v"(st.fm3));
                    if (HLEN) asm volatile("" : "+v"(hlen));
                    asm volatile("" : "+s"(started), "+s"(rare), "+s"(Si));
                }
            }
            // the head began at record 0 (its first contig is ctg[0]); no read
            // starts here: the whole lane is a head
            hd.fm3 = ctg[0] - 3u;
            hd.win = in_mask(started) ? hd.win : st.win;
            // the incoming tail (the previous lane's last read), merged with this
            // lane's head when the read continues (else with itself: the same code)
            const uint64_t t_ok = started & (FULL ? ~0ull : lanes((int)spos < nval));
            const uint32_t t_len = (uint32_t)RPL - spos, t_pos = ubase + spos;
            RState in;
            in.fm3 = dpp_shr1(ct.fm3, st.fm3);
            in.win = dpp_shr1(ct.win, st.win);
            const uint32_t in_pk =
                dpp_shr1(ct_ok ? (ct_len | ct_pos << 8) : kEmpty, in_mask(t_ok) ? (t_len | t_pos << 8) : kEmpty);
            const uint64_t have = lanes(in_pk != kEmpty);
            const uint32_t in_len = in_pk & 255u, in_pos = in_pk >> 8;
            const uint64_t cont = ~S0;
            RState hm;
            hm.fm3 = in_mask(cont) ? hd.fm3 : in.fm3;
            hm.win = in_mask(cont) ? hd.win : in.win;
            uint32_t code, m0;
            const uint64_t ok = rs_code2_m<COMPACT, BIN>(in, hm, P.N, &code, &m0);
            // big: the read runs past this lane (no start in it: its length is
            // unknown here), or has > 8 records.  16 records per lane: a read
            // seen whole (tail alone, or tail + head) is a code when compact,
            // whatever its length, and big only when general and > 8 records
            const uint64_t big =
                RPL > 8 ? (!HLEN ? cont & ~started
                                 : (cont & lanes(hlen == (uint32_t)RPL)) |
                                       (lanes(in_len + (in_mask(cont) ? hlen : 0u) > (uint32_t)kMaxFast) & ~ok))
                        : cont & lanes(in_len + hlen > (uint32_t)kMaxFast);
            emit(have, ok, code, m0, in_pos, big);
            return rare;
        };
        if (REPLAY) {
            RState st2;
            uint32_t spos2;
            uint64_t started2;
            walk(std::true_type{}, st2, spos2, started2);
            return;
        }
        RState st;
        uint32_t spos;
        uint64_t started;
        const uint64_t rare = walk(std::false_type{}, st, spos, started);
        // this lane's tail (an own read reaching its last record) -> the next
        // lane; carry lane 63 into the next step
        const uint64_t t_ok = started & (FULL ? ~0ull : lanes((int)spos < nval));
        const uint32_t t_len = (uint32_t)RPL - spos, t_pos = ubase + spos;
        const bool ct_ok_next = (t_ok >> 63) != 0;
        RState ct_next;
        ct_next.fm3 = (uint32_t)__builtin_amdgcn_readlane((int)st.fm3, 63);
        ct_next.win = (uint32_t)__builtin_amdgcn_readlane((int)st.win, 63);
        const uint32_t ct_len_next = (uint32_t)__builtin_amdgcn_readlane((int)t_len, 63);
        const uint32_t ct_pos_next = (uint32_t)__builtin_amdgcn_readlane((int)t_pos, 63);
        if (RC && BIN) bin_stage();  // (its codes' range test decides the listing too)
        if (KARMA_CLS_DEFER_RARE && (rare || (RC && stage_hi))) {
            // listed with its carry-in (ct* and prev_rid still hold it here)
            if (lane == 0) {
                uint32_t* const e = rl + kRareW * n_rare;
                e[0] = (uint32_t)((t0 - c_lo) / kIt) | (ct_ok ? 256u : 0u) | (have_prev ? 512u : 0u);
                e[1] = ct.fm3;
                e[2] = ct.win;
                e[3] = ct_len | ct_pos << 8;
                e[4] = prev_rid;
            }
            ++n_rare;
        } else if (!KARMA_CLS_DEFER_RARE && !KARMA_CLS_NO_RARE && rare) {
            RState st2;
            uint32_t spos2;
            uint64_t started2;
            walk(std::true_type{}, st2, spos2, started2);
        }
        if (BIN && !RC) bin_stage();  // before the next step's transpose reuses the buffer
        if (RC) stage_hi = 0;
        ct_ok = ct_ok_next;
        ct = ct_next;
        ct_len = ct_len_next;
        ct_pos = ct_pos_next;
        if (!FLAG) prev_rid = (uint32_t)__builtin_amdgcn_readlane((int)rid[RPL - 1], 63);
        have_prev = true;
    };
    u32x4 buf[kCPer];
    prefetch(buf, c_lo, c_hi);
    // the relabel word (set by the probe kernel, or by this kernel's votes:
    // read past the L2 of this XCD), once the chunk's first records are in
    // flight (its latency hides under theirs)
    if (P.skip && __hip_atomic_load(P.skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        if (lane == 0) {
            const ClassArgs& Pa = P;
            Pa.n_codes[chunk] = 0;
            Pa.n_gen[chunk] = 0;
            if (BIN)
                for (int i = 0; i < kBinHdr; ++i) Q.hdr[kBinHdr * chunk + i] = uint4{0u, 0u, 0u, 0u};
        }
        if (BIN && Q.slotted) {  // the reduce reads every slot: empty ones
            const BinArgs& Qa = Q;
            for (uint32_t k = lane; k < (uint32_t)P.Bc * 8u; k += 64)
                *reinterpret_cast<u32x4*>(Qa.segs + (chunk * Qa.seg_cap + (k >> 3)) * kBinQ + 8 * (k & 7u)) =
                    u32x4{~0u, ~0u, ~0u, ~0u};
        }
        return;
    }
    const std::false_type main_pass{};
    if (!REMAP) {
        int64_t t0 = c_lo;
        for (; t0 + kIt <= c_hi; t0 += kIt) step(std::true_type{}, main_pass, buf, buf, t0);
        if (t0 < c_hi) step(std::false_type{}, main_pass, buf, buf, t0);
    } else {  // two register sets, alternating
        u32x4 buf2[kCPer];
        if (c_lo + kIt < c_hi) prefetch(buf2, c_lo + kIt, c_hi);
        remap_units(buf);
        for (int64_t t0 = c_lo; t0 < c_hi;) {
            if (t0 + kIt <= c_hi) step(std::true_type{}, main_pass, buf, buf2, t0);
            else step(std::false_type{}, main_pass, buf, buf2, t0);
            t0 += kIt;
            if (t0 >= c_hi) break;
            if (t0 + kIt <= c_hi) step(std::true_type{}, main_pass, buf2, buf, t0);
            else step(std::false_type{}, main_pass, buf2, buf, t0);
            t0 += kIt;
        }
    }
    if (KARMA_CLS_DEFER_RARE && n_rare) {
        // the listed steps again (in step order: the general starts land in the
        // chunk's region in the order the in-loop pass wrote them), each from
        // its carry-in; the chunk's own carry is restored for the tail below
        const bool s_ok = ct_ok, s_hp = have_prev;
        const RState s_ct = ct;
        const uint32_t s_len = ct_len, s_pos = ct_pos, s_rid = prev_rid;
        wave_lds_order();
        for (uint32_t k = 0; k < n_rare; ++k) {
            const uint32_t* const e = rl + kRareW * k;
            const uint32_t w0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)e[0]);
            ct_ok = (w0 & 256u) != 0;
            have_prev = (w0 & 512u) != 0;
            ct.fm3 = (uint32_t)__builtin_amdgcn_readfirstlane((int)e[1]);
            ct.win = (uint32_t)__builtin_amdgcn_readfirstlane((int)e[2]);
            const uint32_t w3 = (uint32_t)__builtin_amdgcn_readfirstlane((int)e[3]);
            ct_len = w3 & 255u;
            ct_pos = w3 >> 8;
            prev_rid = (uint32_t)__builtin_amdgcn_readfirstlane((int)e[4]);
            const int64_t t0 = c_lo + (int64_t)(w0 & 255u) * kIt;
            prefetch(buf, t0, c_hi);
            if (REMAP) remap_units(buf);
            if (t0 + kIt <= c_hi) step(std::true_type{}, std::true_type{}, buf, buf, t0);
            else step(std::false_type{}, std::true_type{}, buf, buf, t0);
        }
        ct_ok = s_ok;
        have_prev = s_hp;
        ct = s_ct;
        ct_len = s_len;
        ct_pos = s_pos;
        prev_rid = s_rid;
    }
    // the chunk's last tail read continues into the next chunk's first records
    // (at most 8 of them matter): uniform scalar walk
    if (ct_ok) {
        RState h{};
        uint32_t hl = 0;
        for (; hl < (uint32_t)kMaxFast && c_hi + hl < P.A; ++hl) {
            uint32_t y;
            if (FLAG) {
                const uint32_t w = P.recw[c_hi + hl];
                if ((int)w < 0) break;  // the next read starts
                y = w & kContigMask;
            } else {
                const uint2 r = P.rec[c_hi + hl];
                if (r.x != prev_rid) break;
                y = r.y;
            }
            const uint32_t cy = REMAP && y < P.N ? P.remap[y] : y;
            if (hl == 0) rs_reset(h, cy);
            else rs_add(h, cy);
        }
        const bool big = ct_len + hl > (uint32_t)kMaxFast;
        uint32_t code;
        const bool ok = !big && (hl ? rs_code2<COMPACT>(ct, h, P.N, &code) : rs_code<COMPACT>(ct, P.N, &code));
        // lane 0's code (uniform values), in the staged form m0 << 4 | M << 1 | 1
        if (BIN && ok) {
            const uint32_t rel = (code >> 24) << 1 | 1u;
            if (RC && (code & 0xFFFFFFu) + 31u - (uint32_t)__builtin_clz(rel) >= P.N) bad_contig |= 1ull;
            bin_emit(1ull, (code & 0xFFFFFFu) << 4 | rel);
        }
        if (lane == 0) {
            const ClassArgs& Pa = P;
            if (big) Pa.big_list[atomicAdd(Pa.big_n, 1u)] = c_lo + ct_pos;
            else if (ok) {
                if (!BIN) out[nc] = code;
                if (hist_on) atomicAdd(&wh[(code & 0xFFFFFFu) >> P.bwc], 1u);
            } else (BIN ? Pa.codes + c_lo : out)[P.chunk - 1 - ng] = ct_pos;
        }
        nc += ok ? 1u : 0u;
        ng += !big && !ok ? 1u : 0u;
    }
    if (BIN && Q.slotted) {
        // slotted (the queues fill well: >= ~40 codes per bucket and chunk):
        // every bucket's queue as one whole 128-byte segment at slot b of the
        // chunk's region, past its count 0xFFFF.  The reduce then reads each
        // bucket's fronts as aligned 128-byte segments at fixed places
        // (5.7 TB/s in tools/micro/seg_read.hip against 2.8 for ~110-byte
        // runs at hashed offsets); no granule counts in the header
        wave_lds_order();
        const BinArgs& Qa = Q;
        for (uint32_t k = lane; k < (uint32_t)P.Bc * 8u; k += 64) {
            const uint32_t bk = k >> 3, i = k & 7u;
            const uint32_t n = qn[bk];
            u32x4 v = *reinterpret_cast<const u32x4*>(q + bk * kBinQ + 8 * i);
            const int k0c = 8 * (int)i;
            auto pad = [&](uint32_t w, int c) -> uint32_t {
                const uint32_t lo = k0c + c < (int)n ? (w & 0xFFFFu) : 0xFFFFu;
                const uint32_t hi = k0c + c + 1 < (int)n ? (w >> 16) : 0xFFFFu;
                return lo | hi << 16;
            };
            v.x = pad(v.x, 0), v.y = pad(v.y, 2), v.z = pad(v.z, 4), v.w = pad(v.w, 6);
            *reinterpret_cast<u32x4*>(Qa.segs + (chunk * Qa.seg_cap + bk) * kBinQ + 8 * i) = v;
        }
        if (lane == 0) {
            uint4* const h = Q.hdr + kBinHdr * chunk;
            h[0] = uint4{0u, 0u, 0u, 0u};
            h[1] = uint4{0u, 0u, 0u, bst[0]};
            h[2] = uint4{bst[1], bst[2], bst[3], bst[4]};
            h[3] = uint4{bst[5], bst[6], nc, 0u};
        }
    } else if (BIN) {
        // the front runs: every non-empty queue, in bucket order, as 16-byte
        // granules; granule k of the chunk is found through a table in the
        // (now idle) transpose buffer: k -> bucket << 3 | granule
        wave_lds_order();
        const uint32_t cnt = lane < P.Bc ? qn[lane] : 0u;
        const uint32_t g = (cnt + 7u) >> 3;
        const uint32_t incl = wave_scan_incl(g), excl = incl - g;
        const uint32_t G = lane63(incl);
        uint16_t* const gt = reinterpret_cast<uint16_t*>(tb);  // <= 56 x 8 entries
        uint8_t* const gb = reinterpret_cast<uint8_t*>(tb) + 1024;  // granule count per bucket
        for (uint32_t i = 0; i < g; ++i) gt[excl + i] = (uint16_t)(lane << 3 | i);
        gb[lane] = (uint8_t)g;
        wave_lds_order();
        for (uint32_t k0 = 0; k0 < G; k0 += 64) {
            const uint32_t k = k0 + lane;
            if (k < G) {
                const uint32_t e = gt[k], bk = e >> 3, i = e & 7u;
                const uint32_t n = qn[bk];
                u32x4 v = *reinterpret_cast<const u32x4*>(q + bk * kBinQ + 8 * i);
                // codes at index >= n are stale: 0xFFFF
                const int k0c = 8 * (int)i;
                auto pad = [&](uint32_t w, int c) -> uint32_t {
                    const uint32_t lo = k0c + c < (int)n ? (w & 0xFFFFu) : 0xFFFFu;
                    const uint32_t hi = k0c + c + 1 < (int)n ? (w >> 16) : 0xFFFFu;
                    return lo | hi << 16;
                };
                v.x = pad(v.x, 0), v.y = pad(v.y, 2), v.z = pad(v.z, 4), v.w = pad(v.w, 6);
                const BinArgs& Qa = Q;
                *reinterpret_cast<u32x4*>(Qa.segs + chunk * Qa.seg_cap * kBinQ + (int64_t)k * 8) = v;
            }
        }
        // the header: lane w < 7 packs the nibbles of buckets 8w .. 8w + 7
        uint32_t nib = 0;
        if (lane < 7) {
#pragma unroll
            for (int j = 0; j < 8; ++j) nib |= (uint32_t)(8 * lane + j < P.Bc ? gb[8 * lane + j] : 0u) << (4 * j);
        }
        const uint32_t w0 = (uint32_t)__builtin_amdgcn_readlane((int)nib, 0);
        const uint32_t w1 = (uint32_t)__builtin_amdgcn_readlane((int)nib, 1);
        const uint32_t w2 = (uint32_t)__builtin_amdgcn_readlane((int)nib, 2);
        const uint32_t w3 = (uint32_t)__builtin_amdgcn_readlane((int)nib, 3);
        const uint32_t w4 = (uint32_t)__builtin_amdgcn_readlane((int)nib, 4);
        const uint32_t w5 = (uint32_t)__builtin_amdgcn_readlane((int)nib, 5);
        const uint32_t w6 = (uint32_t)__builtin_amdgcn_readlane((int)nib, 6);
        if (lane == 0) {
            uint4* const h = Q.hdr + kBinHdr * chunk;
            h[0] = uint4{w0, w1, w2, w3};
            h[1] = uint4{w4, w5, w6, bst[0]};
            h[2] = uint4{bst[1], bst[2], bst[3], bst[4]};
            h[3] = uint4{bst[5], bst[6], nc, 0u};
        }
    }
    if (lane == 0) {
        const ClassArgs& Pa = P;
        Pa.n_codes[chunk] = nc;
        Pa.n_gen[chunk] = ng;
        if (nc && !BIN) atomicAdd(Pa.blk_items + chunk / Pa.lists_per_block, (unsigned long long)nc);
    }
    if (hist_on && nc) {
        wave_sync();
        uint32_t* gh = P.blk_hist + (chunk / P.lists_per_block) * P.Bc;
        for (int b = lane; b < P.Bc; b += 64) {
            const uint32_t k = wh[b];
            if (k) atomicAdd(gh + b, k);
        }
    }
    if (lane == 0) {
        const ClassArgs& Pa = P;
        if (bad_order) Pa.flags[0] = 1;
        if (bad_contig) Pa.flags[1] = 1;
        // kVotes, or half the voting chunks of a small job
        const int64_t voters = ((Pa.A + Pa.chunk - 1) / Pa.chunk + kVoteStride - 1) / kVoteStride;
        const unsigned need = (unsigned)min<int64_t>(kVotes, (voters + 1) / 2);
        if (Pa.vote && chunk % kVoteStride == 0 && 8 * ng > nc + ng && nc + ng >= 64 &&
            atomicAdd(Pa.vote, 1u) + 1 == need)
            __hip_atomic_store(Pa.skip, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- general reads -----------------------------------------------------------------
constexpr int kGW = 256;  // general-kernel threads (4 waves, one chunk each)
// the general kernel's grid: a wave per chunk up to 4 blocks per CU
int general_grid(const karma_ctx* ctx, int64_t n_chunks) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n_chunks, kGW / 64), (int64_t)ctx->cu_count * 4));
}

// A wave per chunk, grid-stride (the grid is sized to the chip, not to the
// chunk count: on assembled transcriptomes almost every chunk has no general
// read, and dispatching one wave per chunk cost 17-23 us at the 8-rank strong
// preview while the code partition waited for CU slots): every pair (p <= q)
// of each general read's distinct contigs, as (a << 32 | b), appended to the
// chunk's pair list.
__global__ void __launch_bounds__(kGW) general_kernel(RecIn rec, int64_t A, uint32_t N,
                                                       const uint32_t* __restrict__ codes,
                                                       const uint32_t* __restrict__ n_gen, int64_t n_chunks,
                                                       uint64_t* __restrict__ pairs, int64_t pcap,
                                                       uint32_t* __restrict__ n_pairs,
                                                       unsigned long long* __restrict__ blk_items,
                                                       int lists_per_block, int* __restrict__ flags,
                                                       const uint32_t* __restrict__ remap,
                                                       const unsigned* __restrict__ relabel, int64_t chunk_len) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // a relabelled rerun follows (relabel_probe_kernel): no pairs now
    const bool skip = relabel && *relabel;
    for (int64_t chunk = (int64_t)blockIdx.x * (kGW / 64) + wave; chunk < n_chunks;
         chunk += (int64_t)gridDim.x * (kGW / 64)) {
    const uint32_t ng = skip ? 0u : n_gen[chunk];
    uint32_t np = 0;
    uint64_t* out = pairs + chunk * pcap;
    const int64_t c_lo = chunk * chunk_len;
    bool full = false, bad = false;  // bad: a contig >= N (the binned flagged classify checks codes only)
    for (uint32_t kb = 0; kb < ng; kb += 64) {
        const uint32_t k = kb + lane;
        ReadSet rs;
        rs.u = 0;
#pragma unroll
        for (int t = 0; t < kMaxFast; ++t) rs.keep[t] = false;
        if (k < ng) {
            const int64_t s = c_lo + codes[c_lo + chunk_len - 1 - k];
            bool v = true;
#pragma unroll
            for (int t = 0; t < kMaxFast; ++t) {
                v = v && s + t < A && (t == 0 || rec.cont(s + t));
                const uint32_t y = v ? rec.contig(s + t) : kEmpty;
                bad |= v && y >= N;
                rs.m[t] = v && y < N ? (remap ? remap[y] : y) : kEmpty;
            }
            sort_dedup(rs);
        }
        const uint32_t cnt = rs.u * (rs.u + 1) / 2;
        const uint32_t x = wave_scan_incl(cnt);  // wave inclusive scan of the pair counts
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
        if ((int64_t)np + total > pcap) {
            full = true;
            break;
        }
        uint64_t* o = out + np + (x - cnt);
#pragma unroll
        for (int p = 0; p < kMaxFast; ++p) {
            if (!rs.keep[p]) continue;
#pragma unroll
            for (int q = p; q < kMaxFast; ++q)
                if (rs.keep[q]) *o++ = ((uint64_t)rs.m[p] << 32) | rs.m[q];
        }
        np += total;
    }
    if (lane == 0) {
        n_pairs[chunk] = np;
        if (np) atomicAdd(blk_items + chunk / lists_per_block, (unsigned long long)np);
        if (full) flags[2] = 1;  // the host reruns with room for every pair
    }
    if (bad) flags[1] = 1;
    }
}

// ---- partition: chunk lists -> bucket-major padded runs ---------------------------
constexpr int kPT = 512;                 // partition threads (several blocks per CU overlap their phases)
constexpr int kMaxListsPerBlock = 128;   // chunk lists per partition block, at most (a power of 2)

#ifndef KARMA_CODE_FILL
#define KARMA_CODE_FILL 8192  // codes per partition flush (A/B builds: shorter runs for the reduce)
#endif
// compact-read codes: u32 (m0 | M << 24) -> u16 (m0_local << 3 | M) per code bucket
template <int NB>
struct CodeStreamT {
    using S = uint32_t;
    using D = uint16_t;
    static constexpr int kCap = KARMA_CODE_FILL;  // codes per flush (8192: 32 KB of LDS)
    static constexpr int kPad = 8;      // 16 B of u16
    static constexpr int kMaxNb = NB;
    static constexpr D kPadV = 0xFFFF;  // codes are < 2^15
    // 3 blocks of 8 waves per CU (<= 85 VGPRs) for the narrow variant
    static constexpr int kMinWaves = NB <= 128 ? 6 : 1;
    __device__ static int nb(const Geo& g) { return g.Bc; }
    __device__ static uint32_t bucket(S s, const Geo& g) { return (s & 0xFFFFFFu) >> g.bwc; }
    __device__ static D value(S s, const Geo& g) {
        return (D)(((s & 0xFFFFFFu) & ((1u << g.bwc) - 1u)) << 3 | (s >> 24));
    }
};

// general pairs: u64 (a << 32 | b) -> u32 (a_local << bbits | b) per pair bucket
template <int NB>
struct PairStreamT {
    using S = uint64_t;
    using D = uint32_t;
    static constexpr int kCap = 4096;
    static constexpr int kPad = 4;
    static constexpr int kMaxNb = NB;
    static constexpr D kPadV = kEmpty;  // pair keys are < 2^31
    static constexpr int kMinWaves = 1;
    __device__ static int nb(const Geo& g) { return g.B; }
    __device__ static uint32_t bucket(S s, const Geo& g) { return (uint32_t)(s >> 32) >> g.bw; }
    __device__ static D value(S s, const Geo& g) {
        return (((uint32_t)(s >> 32) & ((1u << g.bw) - 1u)) << g.bbits) | (uint32_t)s;
    }
};

using CodeStream = CodeStreamT<kNarrowBc>;
using CodeStreamWide = CodeStreamT<kMaxBc>;
using PairStream = PairStreamT<kNarrowB>;
using PairStreamWide = PairStreamT<kMaxB>;

struct RunDir {
    int64_t* base;                        // per flush: start of its runs in the stream
    uint32_t* off;                        // per flush: nb + 1 run offsets
    unsigned* n;                          // flushes (directory rows) in all
    const unsigned long long* blk_items;  // per partition block: items (from the producers)
};

// A buffer resource over [base, base + bytes) from block-uniform values (read
// from the first lane), for stores whose out-of-range lanes are dropped.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, uint32_t bytes) {
    const uint64_t u = (uint64_t)base;
    return __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(u >> 32)) << 32) |
                                (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u)),
        0, (int)(uint32_t)__builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}

// N vector stores that the range check drops (an empty buffer resource;
// volatile, so none is merged away)
template <int N>
__device__ __forceinline__ void dropped_stores() {
    const __amdgpu_buffer_rsrc_t none = __builtin_amdgcn_make_buffer_rsrc(nullptr, 0, 0, 0x00020000);
#pragma unroll
    for (int t = 0; t < N; ++t) __builtin_amdgcn_raw_buffer_store_b32(0u, none, 4 * t, 0, 1 << 31);
}

// A partition block's items (blk_items, summed by the producers), flushes
// (every flush but the last holds cap items) and an output bound (items + <
// pad per run): the bases of block b are these sums over blocks < b, so each
// block derives its own directory rows and stream slice (no atomics, no plan
// launch).
__device__ __forceinline__ void part_need(uint64_t items, int cap, int nb, int pad, int64_t* outs, int64_t* rows) {
    *rows = ((int64_t)items + cap - 1) / cap;
    *outs = ((int64_t)items + *rows * (int64_t)nb * (pad - 1) + pad - 1) / pad * pad;
}

template <class T>
__global__ void __launch_bounds__(kPT) __attribute__((amdgpu_waves_per_eu(T::kMinWaves)))
partition_kernel(const typename T::S* __restrict__ lists, int64_t list_cap,
                                                         const uint32_t* __restrict__ list_n, int64_t n_lists,
                                                         int per_block, Geo g, typename T::D* __restrict__ out,
                                                         RunDir dir) {
    using S = typename T::S;
    using D = typename T::D;
    constexpr int kPer = T::kCap / kPT;  // items per thread per fill
    constexpr int kVMax = (T::kCap + T::kMaxNb * (T::kPad - 1)) * (int)sizeof(D) / 16;  // vectors per flush, at most
    constexpr int kCopyIt = (kVMax + kPT - 1) / kPT;
    __shared__ S buf[T::kCap];
    __shared__ D sorted[T::kCap + T::kMaxNb * (T::kPad - 1)];
    // Per-bucket counters.  Each item's add returns its rank among the fill's
    // items of its bucket, kept in registers; the flush's scan turns the
    // counts into run offsets (toff), writes the runs' padding and clears the
    // counts, and the scatter is a plain LDS store at toff[b] + rank (round 3:
    // one LDS atomic per item instead of two; the cursor adds had repeated
    // the count adds' same-address conflicts).
    __shared__ uint32_t hist[T::kMaxNb];
    __shared__ uint32_t toff[T::kMaxNb + 1];
    __shared__ uint32_t lpre[kMaxListsPerBlock + 1];
    __shared__ int64_t red_s[2][kPT / 64];
    const int nb = T::nb(g);
    int64_t used = 0;  // stream items of this block's flushes so far (uniform)
    int row = 0;       // directory rows of this block so far (uniform)
    int64_t out0, row0;  // this block's stream slice and first directory row
    {
        int64_t so = 0, sr = 0;
        for (int64_t b = threadIdx.x; b < (int64_t)blockIdx.x; b += kPT) {
            int64_t o, r;
            part_need(dir.blk_items[b], T::kCap, nb, T::kPad, &o, &r);
            so += o;
            sr += r;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            so += __shfl_xor(so, d);
            sr += __shfl_xor(sr, d);
        }
        if ((threadIdx.x & 63) == 0) {
            red_s[0][threadIdx.x >> 6] = so;
            red_s[1][threadIdx.x >> 6] = sr;
        }
        __syncthreads();
        out0 = row0 = 0;
        for (int w = 0; w < kPT / 64; ++w) {
            out0 += red_s[0][w];
            row0 += red_s[1][w];
        }
        if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {  // the last block knows the row total
            int64_t o, r;
            part_need(dir.blk_items[blockIdx.x], T::kCap, nb, T::kPad, &o, &r);
            *dir.n = (unsigned)(row0 + r);
        }
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int b = threadIdx.x; b < T::kMaxNb; b += kPT) hist[b] = 0;

    // the block's lists as one concatenated range: prefix of their lengths
    const int64_t l_lo = (int64_t)blockIdx.x * per_block;
    const int nl = (int)min<int64_t>(per_block, n_lists - l_lo);
    if (wave == 0) {
        uint32_t carry = 0;
        for (int base = 0; base < nl; base += 64) {
            const uint32_t v = base + lane < nl ? list_n[l_lo + base + lane] : 0u;
            const uint32_t x = wave_scan_incl(v);
            if (base + lane < nl) lpre[base + lane] = carry + x - v;
            carry += lane63(x);
        }
        for (int i = nl + lane; i <= kMaxListsPerBlock; i += 64) lpre[i] = carry;  // pad: fixed-step search
    }
    __syncthreads();
    const uint32_t items = lpre[nl];
    // items [base, base + kCap) of the range into registers (thread t: t + k * kPT)
    S v[kPer];
    auto load = [&](uint32_t base) {
        // the thread's items rise with k: one fixed-step search for the first,
        // then forward steps (lists hold ~2.7K codes, items are kPT apart)
        int lo = 0;
        {
            const uint32_t g0 = base + threadIdx.x;
#pragma unroll
            for (int step = kMaxListsPerBlock / 2; step >= 1; step >>= 1)
                if (lpre[lo + step] <= g0) lo += step;
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const uint32_t gi = base + threadIdx.x + k * kPT;
            if (gi < items) {
                while (lpre[lo + 1] <= gi) ++lo;  // list L: lpre[L] <= gi < lpre[L + 1]
                if (KARMA_PART_LOAD_NT)
                    v[k] = __builtin_nontemporal_load(&lists[(l_lo + lo) * list_cap + (gi - lpre[lo])]);
                else
                    v[k] = lists[(l_lo + lo) * list_cap + (gi - lpre[lo])];
            }
        }
    };
    load(0);
    // every path into the flush loop has kCopyIt stores after the fill's loads
    // (here dropped ones), so the loop's wait for a fill stays vmcnt(kCopyIt)
    dropped_stores<kCopyIt>();
    // a thread scatters the items it counted (its own slots of the fill),
    // staged in LDS across the flush's barriers while v takes the next
    // fill's loads (held in registers instead: 104 VGPRs, 2 blocks per CU,
    // measured slower)
#define PART_ITEM(k) buf[threadIdx.x + (k) * kPT]
    for (uint32_t base = 0; base < items; base += T::kCap) {
        const uint32_t n = min(items - base, (uint32_t)T::kCap);
        uint32_t rk[(kPer + 1) / 2];  // ranks within the bucket, two 16-bit ranks per register
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const uint32_t i = threadIdx.x + k * kPT;
            PART_ITEM(k) = v[k];
            const uint32_t r = i < n ? atomicAdd(&hist[T::bucket(v[k], g)], 1u) : 0u;
            if (k & 1) rk[k >> 1] |= r << 16;
            else rk[k >> 1] = r;
        }
        load(base + T::kCap);  // the next fill's loads overlap this flush
        // ---- flush: counting sort of buf by bucket into padded runs ----
        __syncthreads();
        if (wave == 0) {
            uint32_t c2 = 0;
            for (int b0 = 0; b0 < nb; b0 += 64) {
                const int bb = b0 + lane;
                const uint32_t cnt = bb < nb ? hist[bb] : 0u;
                if (bb < nb) hist[bb] = 0;  // counted: clear for the next fill
                const uint32_t val = (cnt + (T::kPad - 1)) & ~(uint32_t)(T::kPad - 1);
                const uint32_t x = wave_scan_incl(val);
                if (bb < nb) {
                    const uint32_t o = c2 + x - val;
                    toff[bb] = o;
                    for (uint32_t i = o + cnt; i < c2 + x; ++i) sorted[i] = T::kPadV;  // the run's padding
                }
                c2 += lane63(x);
            }
            if (lane == 0) toff[nb] = c2;
        }
        __syncthreads();
        const unsigned f = (unsigned)(row0 + row);
        const int64_t at = out0 + used;
        const uint32_t total = toff[nb];
        if (threadIdx.x == 0) dir.base[f] = at;
        ++row;
        used += total;
        {
            for (int b = threadIdx.x; b <= nb; b += kPT) dir.off[(int64_t)f * (nb + 1) + b] = toff[b];
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                if (threadIdx.x + k * kPT < n) {
                    const S it = PART_ITEM(k);
                    const uint32_t r = (rk[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                    sorted[toff[T::bucket(it, g)] + r] = T::value(it, g);
                }
            }
#undef PART_ITEM
        }
        __syncthreads();
        // the counters are clear (scan) and the cursors spent: the next fill
        // may start once this block's 16-byte stores are issued (their
        // completion is never waited for).  Copy-out: a fixed number of 16-byte buffer stores per thread, the
        // range check dropping those past the flush.  vmcnt counts loads and
        // stores together, in issue order: with a runtime-length copy loop the
        // next fill's wait for its (earlier) loads was vmcnt(0) and drained
        // this flush's stores; with a fixed count it is vmcnt(kCopyIt).
        const uint32_t nv = total * (uint32_t)sizeof(D) / 16u;
        const __amdgpu_buffer_rsrc_t drs = uniform_rsrc(out + at, nv * 16u);
        const u32x4* src = reinterpret_cast<const u32x4*>(sorted);
#pragma unroll
        for (int r = 0; r < kCopyIt; ++r) {
            const uint32_t i = threadIdx.x + r * kPT;
            __builtin_amdgcn_raw_buffer_store_b128(src[min(i, (uint32_t)kVMax - 1u)], drs, (int)(i * 16u), 0, 0);
        }
    }
}

// ---- code partition: one run per (block, code bucket) ------------------------------
// The general partition above pads every bucket's run of every flush: with
// hundreds of code buckets (n_contigs > 2^19, the 8-rank weak-scaled config 3)
// a flush's runs hold ~20 codes and the reduce spends its time on run tables.
// Here the classify kernel has already counted each partition block's codes
// per bucket (blk_hist), so a block knows its final run for every bucket up
// front and appends each flush's sorted segment to it: one directory row per
// block, runs of items / Bc codes, padded once.
__device__ __forceinline__ int64_t append_need(uint64_t items, int nb) {
    return ((int64_t)items + (int64_t)nb * 7 + 7) / 8 * 8;
}

// Block barrier for LDS hand-offs only: outstanding global stores and loads are
// not waited for (__syncthreads' release fence would drain vmcnt every flush).
__device__ __forceinline__ void lds_barrier() {
#ifdef KARMA_APPEND_FENCE
    __syncthreads();
#else
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
}

template <int NB>
__global__ void __launch_bounds__(kPT) code_append_kernel(const uint32_t* __restrict__ lists, int64_t list_cap,
                                                           const uint32_t* __restrict__ list_n, int64_t n_lists,
                                                           int per_block, Geo g, const uint32_t* __restrict__ blk_hist,
                                                           uint16_t* __restrict__ out, uint16_t* trash, RunDir dir,
                                                           int* err) {
    using T = CodeStreamT<NB>;
    // codes per flush: 34 KB (narrow) / 79 KB (wide) of LDS, 4 / 2 blocks per CU;
    // wide flushes of 8192 codes write ~20 codes per run instead of ~10
    // (weak-scaled config 3: 0.26-0.27 vs 0.29 ms); 12288: ~30 per run, weak
    // 8-rank preview 1.412 -> 1.397 ms; 16384 leaves one block per CU: 1.60 ms
#ifndef KARMA_APPEND_WIDE_CAP
#define KARMA_APPEND_WIDE_CAP 12288
#endif
    constexpr int kCap = NB > 128 ? KARMA_APPEND_WIDE_CAP : 4096;
    constexpr int kPer = kCap / kPT;
    constexpr int kVMax = kCap / 8 + NB;               // 16-byte vectors of one flush, at most
    constexpr int kVPer = (kVMax + kPT - 1) / kPT;
    // a flush's codes by bucket: bucket b's pending tail (< 8 codes from earlier
    // flushes) then its new codes, from an 8-aligned start toff[b]
    __shared__ __attribute__((aligned(16))) uint16_t s16[kCap + 8 * NB];
    __shared__ __attribute__((aligned(16))) uint16_t pend[8 * NB];
    __shared__ uint32_t hist[2][NB + 1];
    __shared__ uint32_t toff[NB + 1];  // 8-aligned region starts in s16
    __shared__ uint32_t qoff[NB + 1];  // full vectors before bucket b
    __shared__ uint32_t cur[NB];
    __shared__ uint32_t rb[NB + 1];    // the block's run starts in its slice (multiples of 8)
    __shared__ uint32_t wr[NB];        // codes written to run b (multiple of 8)
    __shared__ uint32_t pc[NB];        // pending codes of run b (< 8)
    __shared__ uint32_t dlt[NB];       // slice position of s16[i] (bucket b) = dlt[b] + i
    __shared__ uint16_t vb[kVMax];     // bucket of each full vector of the flush
    __shared__ uint32_t lpre[kMaxListsPerBlock + 1];
    __shared__ int64_t red_s[kPT / 64];
    const int nb = g.Bc;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    {
        int64_t so = 0;
        for (int64_t b = threadIdx.x; b < (int64_t)blockIdx.x; b += kPT) so += append_need(dir.blk_items[b], nb);
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) so += __shfl_xor(so, d);
        if (lane == 0) red_s[wave] = so;
        if (blockIdx.x == 0 && threadIdx.x == 0) *dir.n = gridDim.x;
    }
    const uint32_t* bh = blk_hist + (int64_t)blockIdx.x * nb;
    for (int b = threadIdx.x; b <= nb; b += kPT) hist[0][b] = hist[1][b] = 0;
    for (int b = threadIdx.x; b < nb; b += kPT) wr[b] = pc[b] = 0;
    const int64_t l_lo = (int64_t)blockIdx.x * per_block;
    const int nl = (int)min<int64_t>(per_block, n_lists - l_lo);
    if (wave == 0) {
        // run starts: exclusive scan of the padded per-bucket counts
        uint32_t c2 = 0;
        for (int b0 = 0; b0 < nb; b0 += 64) {
            const uint32_t val = b0 + lane < nb ? (bh[b0 + lane] + 7u) & ~7u : 0u;
            const uint32_t x = wave_scan_incl(val);
            if (b0 + lane < nb) rb[b0 + lane] = c2 + x - val;
            c2 += lane63(x);
        }
        if (lane == 0) rb[nb] = c2;
    } else if (wave == 1) {
        uint32_t carry = 0;
        for (int base = 0; base < nl; base += 64) {
            const uint32_t v = base + lane < nl ? list_n[l_lo + base + lane] : 0u;
            const uint32_t x = wave_scan_incl(v);
            if (base + lane < nl) lpre[base + lane] = carry + x - v;
            carry += lane63(x);
        }
        for (int i = nl + lane; i <= kMaxListsPerBlock; i += 64) lpre[i] = carry;
    }
    __syncthreads();
    int64_t out0 = 0;
    for (int w = 0; w < kPT / 64; ++w) out0 += red_s[w];
    if (threadIdx.x == 0) dir.base[blockIdx.x] = out0;
    for (int b = threadIdx.x; b <= nb; b += kPT) dir.off[(int64_t)blockIdx.x * (nb + 1) + b] = rb[b];
    const uint32_t items = lpre[nl];
    u32x4* const vout = reinterpret_cast<u32x4*>(out + out0);  // out0 is a multiple of 8
    u32x4* const vtrash = reinterpret_cast<u32x4*>(trash);
    uint32_t v[kPer];
    // Loads and stores of the flush loop are unconditional (clamped loads, stores
    // past the end go to `trash`): the compiler then counts them exactly and the
    // next fill waits for its loads only, not for the stores issued after them.
    auto load = [&](uint32_t base) {
        int lo = 0;
        {
            const uint32_t g0 = min(base + threadIdx.x, items - 1);
#pragma unroll
            for (int step = kMaxListsPerBlock / 2; step >= 1; step >>= 1)
                if (lpre[lo + step] <= g0) lo += step;
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const uint32_t gi = min(base + threadIdx.x + k * kPT, items - 1);
            while (lpre[lo + 1] <= gi) ++lo;
            v[k] = KARMA_APPEND_LOAD_NT ? __builtin_nontemporal_load(&lists[(l_lo + lo) * list_cap + (gi - lpre[lo])])
                                        : lists[(l_lo + lo) * list_cap + (gi - lpre[lo])];
        }
    };
    if (items > 0) load(0);
    int parity = 0;
    uint32_t x[kPer];  // this thread's items of the flush (it scatters what it counted)
    for (uint32_t base = 0; base < items; base += kCap, parity ^= 1) {
        const uint32_t n = min(items - base, (uint32_t)kCap);
        uint32_t* h = hist[parity];
        uint32_t rk[(kPer + 1) / 2];  // ranks within the bucket (as in partition_kernel), two per register
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const uint32_t i = threadIdx.x + k * kPT;
            x[k] = v[k];
            const uint32_t r = i < n ? atomicAdd(&h[T::bucket(x[k], g)], 1u) : 0u;
            if (k & 1) rk[k >> 1] |= r << 16;
            else rk[k >> 1] = r;
        }
        load(base + kCap);
        lds_barrier();
        // bucket regions (pending + new, 8-aligned), full-vector counts and
        // the scatter cursors (region start + pending codes)
        if (wave == 0) {
            uint32_t c8 = 0, cq = 0;
            for (int b0 = 0; b0 < nb; b0 += 64) {
                const uint32_t tot = b0 + lane < nb ? pc[b0 + lane] + h[b0 + lane] : 0u;
                const uint32_t r8 = (tot + 7u) & ~7u, q = tot >> 3;
                const uint32_t sx = wave_scan_incl(r8), sy = wave_scan_incl(q);
                if (b0 + lane < nb) {
                    toff[b0 + lane] = c8 + sx - r8;
                    qoff[b0 + lane] = cq + sy - q;
                    cur[b0 + lane] = c8 + sx - r8 + pc[b0 + lane];
                }
                c8 += lane63(sx);
                cq += lane63(sy);
            }
            if (lane == 0) toff[nb] = c8, qoff[nb] = cq;
        }
        lds_barrier();
        for (int b = threadIdx.x; b < nb; b += kPT) {
            const uint32_t t = toff[b], p = pc[b];
            // the pending tail: one 16-byte read, then only its p codes (new codes
            // of this bucket land right behind them, concurrently)
            if (p) {
                const u32x4 pv = *reinterpret_cast<const u32x4*>(pend + 8 * b);
                const uint32_t w[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
                for (uint32_t j = 0; j < 7; ++j)
                    if (j < p) s16[t + j] = (uint16_t)(w[j >> 1] >> (16 * (j & 1)));
            }
            for (uint32_t q = qoff[b]; q < qoff[b + 1]; ++q) vb[q] = (uint16_t)b;
            dlt[b] = rb[b] + wr[b] - t;
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            if (threadIdx.x + k * kPT < n) {
                const uint32_t b = T::bucket(x[k], g);
                s16[cur[b] + ((rk[k >> 1] >> (16 * (k & 1))) & 0xFFFFu)] = T::value(x[k], g);
            }
        }
        lds_barrier();
        // full vectors to the runs; the rest of each bucket becomes its pending tail
        const uint32_t nv = qoff[nb];
#pragma unroll
        for (int k = 0; k < kVPer; ++k) {
            const uint32_t t = threadIdx.x + k * kPT;
            const uint32_t b = t < nv ? vb[t] : 0u;
            const uint32_t si = t < nv ? toff[b] + 8u * (t - qoff[b]) : 0u;
            const u32x4 val = *reinterpret_cast<const u32x4*>(s16 + si);
            *(t < nv ? vout + ((dlt[b] + si) >> 3) : vtrash) = val;
        }
        for (int b = threadIdx.x; b < nb; b += kPT) {
            const uint32_t tot = pc[b] + h[b], full = tot & ~7u, r = tot & 7u;
            if (r) *reinterpret_cast<u32x4*>(pend + 8 * b) = *reinterpret_cast<const u32x4*>(s16 + toff[b] + full);
            pc[b] = r;
            wr[b] += full;
            h[b] = 0;
        }
    }
    lds_barrier();
    // the runs' last vectors, padded; the counts must agree with the classify's
    for (int b = threadIdx.x; b < nb; b += kPT) {
        const uint32_t p = pc[b];
        if (wr[b] + p != bh[b]) *err = 1;
        if (p) {
            for (uint32_t j = p; j < 8; ++j) pend[8 * b + j] = T::kPadV;
            vout[(rb[b] + wr[b]) >> 3] = *reinterpret_cast<const u32x4*>(pend + 8 * b);
        }
    }
}

// ---- run streams ------------------------------------------------------------------
// A reduce block reads the runs of one bucket from a range of flushes.  Each
// wave takes batches of 64 runs (lane i holds run i) and reads them as one
// stream of 16-byte vectors, 64 consecutive vectors per load; the runs a
// window of 64 overlaps are found with wave-uniform (scalar) loops over the
// lanes' run table, and kWin windows are in flight before they are counted.
constexpr int kWin = 16;

// slots: 64 ints of LDS per wave of the block.
template <typename Bounds, typename Count>
__device__ __forceinline__ void stream_runs(const u32x4* __restrict__ data, int64_t r_lo, int64_t r_hi, int threads,
                                            Bounds bounds, Count count, const int* stop, int* slots) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int* const wslot = slots + wave * 64;
    // stop == nullptr: nothing stops the block early, so the waves run without
    // a barrier per batch, and the next batch's run bounds are loaded before
    // the current batch is streamed (their latency hides under its windows)
    const bool pipe = KARMA_CR_PIPE && stop == nullptr;
    int64_t nbeg = 0;
    uint32_t nlen = 0;
    if (pipe && r_lo + (int64_t)wave * 64 + lane < r_hi) bounds(r_lo + (int64_t)wave * 64 + lane, &nbeg, &nlen);
    for (int64_t r0 = r_lo + (int64_t)wave * 64; r0 - (int64_t)wave * 64 < r_hi; r0 += (int64_t)threads) {
        const int64_t r = r0 + lane;
        int64_t beg = 0;
        uint32_t len = 0;
        if (pipe) {
            beg = nbeg, len = nlen;
            nbeg = 0, nlen = 0;
            if (r + threads < r_hi) bounds(r + threads, &nbeg, &nlen);
        } else if (r < r_hi) {
            bounds(r, &beg, &len);
        }
        const uint32_t incl = wave_scan_incl(len);
        const uint32_t excl = incl - len;
        const int64_t roff = beg - (int64_t)excl;  // vector j of run r: data[roff + j]
        const uint32_t Tn = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        // the run (lane) holding vector j of a window: each run starting inside
        // the window writes its lane to the window slot of its first vector,
        // then a max-scan over the slots (seeded with the run that covers the
        // previous window's last vector) gives every lane its run
        int carry = -1;
        for (uint32_t j0 = 0; j0 < Tn; j0 += 64u * kWin) {
            u32x4 e[kWin];
#pragma unroll
            for (int u = 0; u < kWin; ++u) {
                const uint32_t w0 = j0 + 64u * u, j = w0 + lane;
                if (w0 >= Tn) continue;  // uniform
                wslot[lane] = -1;
                wave_lds_order();
                if (len && excl >= w0 && excl < w0 + 64u) wslot[excl - w0] = lane;
                wave_lds_order();
                const int rr = wave_max_incl(max(wslot[lane], carry));
                carry = __builtin_amdgcn_readlane(rr, 63);
                const int64_t off = (int64_t)(((uint64_t)(uint32_t)__shfl((int)((uint64_t)roff >> 32), rr) << 32) |
                                              (uint32_t)__shfl((int)(uint32_t)roff, rr));
                if (j < Tn) e[u] = KARMA_RED_LOAD_NT ? __builtin_nontemporal_load(&data[off + j]) : data[off + j];
            }
#pragma unroll
            for (int u = 0; u < kWin; ++u)
                if (j0 + 64u * u + lane < Tn) count(e[u]);
        }
        if (pipe) {
            if (r0 + threads >= r_hi) break;  // this wave's last batch
        } else if (__syncthreads_or(stop != nullptr && *stop != 0)) {
            return;
        }
    }
}

// flushes [f_lo, f_hi) of group `grp` when n_flush (device) is split into n_groups
__device__ __forceinline__ void group_range(const unsigned* n_flush, int n_groups, int grp, int64_t* f_lo,
                                            int64_t* f_hi) {
    const int64_t nf = *n_flush;
    const int64_t per = (nf + n_groups - 1) / n_groups;
    *f_lo = min(nf, grp * per);
    *f_hi = min(nf, *f_lo + per);
}

// ---- code reduce --------------------------------------------------------------------
constexpr int kCRT = 1024;
constexpr int kHistMax = 1 << (kMaxBwCompact + 2 + 3);  // 32768 counters (128 KB)

// One block per (code bucket, group of flushes): histogram of (m0_local, M).
__global__ void __launch_bounds__(kCRT) code_reduce_kernel(const uint16_t* __restrict__ cent, RunDir dir, int Bc,
                                                           int bwc, int n_cg, uint32_t* __restrict__ part_ch) {
    __shared__ uint32_t h[kHistMax];
    __shared__ int slots[kCRT];
    const int bucket = blockIdx.x / n_cg, grp = blockIdx.x % n_cg;
    const int hn = 1 << (bwc + 3);
    for (int i = threadIdx.x; i < hn; i += kCRT) h[i] = 0;
    __syncthreads();
    int64_t f_lo, f_hi;
    group_range(dir.n, n_cg, grp, &f_lo, &f_hi);
    // rows hold one long run per bucket (code_append_kernel): split each into S
    // pieces so that every wave has runs to stream
    const int64_t R = f_hi - f_lo;
    const int S = R > 0 ? (int)max<int64_t>(1, min<int64_t>(KARMA_CR_SMAX, (KARMA_CR_PIECES + R - 1) / R)) : 1;
    // LDS slot of counter c = (m0_local << 3 | M): the low five bits XOR-ed with
    // m0_local >> 2, so that codes of one wave instruction spread over all 32
    // banks (unswizzled, the bank is (m0 & 3) << 3 | M, and M is mostly 0)
    auto slot = [](uint32_t c) { return c ^ ((c >> 5) & 31u); };
    auto add = [&](uint32_t c) {
        if (c != CodeStream::kPadV)
            __hip_atomic_fetch_add(&h[slot(c)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    stream_runs(
        reinterpret_cast<const u32x4*>(cent), f_lo * S, f_hi * S, kCRT,
        [&](int64_t v, int64_t* beg, uint32_t* len) {
            const int64_t f = v / S;
            const uint32_t s = (uint32_t)(v - f * S);
            const uint32_t* o = dir.off + f * (Bc + 1) + bucket;
            const uint32_t L = (o[1] - o[0]) >> 3, seg = (L + S - 1) / S;
            const uint32_t lo = min(L, s * seg), hi = min(L, lo + seg);
            *beg = ((dir.base[f] + o[0]) >> 3) + lo;
            *len = hi - lo;
        },
        [&](const u32x4 v) {
            add(v.x & 0xFFFFu), add(v.x >> 16), add(v.y & 0xFFFFu), add(v.y >> 16);
            add(v.z & 0xFFFFu), add(v.z >> 16), add(v.w & 0xFFFFu), add(v.w >> 16);
        },
        nullptr, slots);
    __syncthreads();
    uint32_t* out = part_ch + (int64_t)blockIdx.x * hn;
    for (int i = threadIdx.x; i < hn; i += kCRT) out[i] = h[slot(i)];
}

// One block per (code bucket, group of chunks) of the binned classify: the
// bucket's runs of the group's chunks into the same direct-mapped LDS
// histogram (same part_ch layout as code_reduce_kernel).
//   front runs   one per chunk (its granule count and offset from the header's
//                nibbles), streamed with stream_runs: batches of 64 chunks,
//                the next batch's headers in flight while one is counted;
//   back segments (a queue that filled mid-chunk; ~10 % of the chunks at
//                config 3) found from the header's first 16 directory bytes
//                (the directory array past them), read 8 per load
//                instruction (8 lanes x 16 B).
__device__ __forceinline__ uint32_t nibble_sum(uint32_t x) {  // sum of the 8 nibbles
    x = (x & 0x0F0F0F0Fu) + ((x >> 4) & 0x0F0F0F0Fu);
    return (x * 0x01010101u) >> 24;
}
constexpr int kBackList = 2048;  // chunks with back segments of the block's bucket, listed in LDS
__global__ void __launch_bounds__(kCRT) code_seg_reduce_kernel(const uint16_t* __restrict__ segs,
                                                               const uint4* __restrict__ hdr,
                                                               const uint8_t* __restrict__ dir, int64_t n_chunks,
                                                               uint32_t seg_cap, int dir_cap, int bwc, int n_cg,
                                                               uint32_t* __restrict__ part_ch, uint32_t list_cap,
                                                               int slotted) {
    __shared__ uint32_t h[kHistMax];
    __shared__ int slots[kCRT];
    __shared__ uint32_t blist[kBackList];
    __shared__ uint32_t nlist;
    const int bucket = blockIdx.x / n_cg, grp = blockIdx.x % n_cg;
    const int hn = 1 << (bwc + 3);
    for (int i = threadIdx.x; i < hn; i += kCRT) h[i] = 0;
    if (threadIdx.x == 0) nlist = 0;
    __syncthreads();
    const int64_t per = (n_chunks + n_cg - 1) / n_cg;
    const int64_t c_lo = min(n_chunks, (int64_t)grp * per), c_hi = min(n_chunks, c_lo + per);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    auto slot = [](uint32_t c) { return c ^ ((c >> 5) & 31u); };
    auto add = [&](uint32_t c) {
        if (c != 0xFFFFu) __hip_atomic_fetch_add(&h[slot(c)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto add8 = [&](const u32x4 v) {
        add(v.x & 0xFFFFu), add(v.x >> 16), add(v.y & 0xFFFFu), add(v.y >> 16);
        add(v.z & 0xFFFFu), add(v.z >> 16), add(v.w & 0xFFFFu), add(v.w >> 16);
    };
    const int bw_ = bucket >> 3, bs = 4 * (bucket & 7);
    auto list_back = [&](int64_t c, uint32_t bmw) {  // a chunk whose back mask holds the bucket
        if ((bmw >> (bucket & 31)) & 1u) {
            const uint32_t i = __hip_atomic_fetch_add(&nlist, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (i < list_cap) blist[i] = (uint32_t)(c - c_lo);
        }
    };
    if (slotted) {
        // front slot `bucket` of every chunk: whole 128-byte segments at fixed
        // places, 8 lanes each, 8 per load instruction; the next 64 chunks'
        // segments are loaded while these are counted (two register sets);
        // lane l also reads chunk c0 + l's back mask
        auto load = [&](u32x4 (&v)[8], int64_t c0) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int64_t c = c0 + 8 * t + (lane >> 3);
                if (c < c_hi)
                    v[t] = *reinterpret_cast<const u32x4*>(segs + ((int64_t)c * seg_cap + bucket) * kBinQ + 8 * (lane & 7));
            }
        };
        auto count = [&](const u32x4 (&v)[8], int64_t c0) {
            if (c0 + lane < c_hi) {
                const uint4 h2 = hdr[kBinHdr * (c0 + lane) + 2];
                list_back(c0 + lane, bucket < 32 ? h2.x : h2.y);
            }
#pragma unroll
            for (int t = 0; t < 8; ++t)
                if (c0 + 8 * t + (lane >> 3) < c_hi) add8(v[t]);
        };
        u32x4 va[8], vb[8];
        int64_t c0 = c_lo + (int64_t)wave * 64;
        if (c0 < c_hi) load(va, c0);
        while (c0 < c_hi) {
            if (c0 + kCRT < c_hi) load(vb, c0 + kCRT);
            count(va, c0);
            c0 += kCRT;
            if (c0 >= c_hi) break;
            if (c0 + kCRT < c_hi) load(va, c0 + kCRT);
            count(vb, c0);
            c0 += kCRT;
        }
    } else
    // front runs: run r = chunk r's granules of this bucket; a chunk whose
    // back mask holds the bucket is listed for the back pass on the way
    stream_runs(
        reinterpret_cast<const u32x4*>(segs), c_lo, c_hi, kCRT,
        [&](int64_t c, int64_t* beg, uint32_t* len) {
            const uint4 h0 = hdr[kBinHdr * c], h1 = hdr[kBinHdr * c + 1], h2 = hdr[kBinHdr * c + 2];
            const uint32_t w[7] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z};
            uint32_t pre = 0, mine = 0;
#pragma unroll
            for (int i = 0; i < 7; ++i) {
                pre += i < bw_ ? nibble_sum(w[i]) : 0u;
                if (i == bw_) {
                    pre += nibble_sum(w[i] & ((1u << bs) - 1u));
                    mine = (w[i] >> bs) & 15u;
                }
            }
            *beg = c * (int64_t)seg_cap * (kBinQ / 8) + pre;
            *len = mine;
            list_back(c, bucket < 32 ? h2.x : h2.y);
        },
        add8, nullptr, slots);
    __syncthreads();
    // back segments of the listed chunks (every chunk of the group when the
    // list overflowed: a skewed input), a chunk per lane
    uint32_t* const wt = reinterpret_cast<uint32_t*>(slots) + wave * 64;
    auto stream8 = [&](uint64_t m, uint32_t seg) {  // one whole segment per lane in m
        const int n = __popcll(m);
        wave_lds_order();
        if (in_mask(m)) wt[rank_below(m)] = seg;
        wave_lds_order();
        u32x4 v[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int j = 8 * t + (lane >> 3);
            if (8 * t < n && j < n) v[t] = *reinterpret_cast<const u32x4*>(segs + (int64_t)wt[j] * kBinQ + 8 * (lane & 7));
        }
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (8 * t < n && 8 * t + (lane >> 3) < n) add8(v[t]);
    };
    const uint8_t bb = (uint8_t)bucket;
    const uint32_t nl = nlist;
    const bool listed = nl <= list_cap;
    const int64_t n_items = listed ? (int64_t)nl : c_hi - c_lo;
    for (int64_t i0 = (int64_t)wave * 64; i0 < n_items; i0 += kCRT) {
        const int64_t i = i0 + lane;
        const int64_t c = i < n_items ? c_lo + (listed ? (int64_t)blist[i] : i) : c_hi;
        uint4 h1 = {0u, 0u, 0u, 0u}, h2 = {0u, 0u, 0u, 0u}, h3 = {0u, 0u, 0u, 0u};
        if (c < c_hi) {
            h2 = hdr[kBinHdr * c + 2];
            h1 = hdr[kBinHdr * c + 1];
            h3 = hdr[kBinHdr * c + 3];
        }
        const uint64_t bm = h2.x | (uint64_t)h2.y << 32;
        uint64_t mb = lanes((bm >> bucket) & 1ull);
        if (!mb) continue;
        const uint32_t nb = h1.w;
        // matches among the first 16 directory bytes
        const uint32_t d[4] = {h2.z, h2.w, h3.x, h3.y};
        uint32_t hit = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            hit |= (((d[k >> 2] >> (8 * (k & 3))) & 0xFFu) == bb && (uint32_t)k < nb) ? 1u << k : 0u;
        for (uint32_t base = 0;;) {
            // this lane's matches in [base, base + 16), one segment per round
            for (;;) {
                const uint64_t mm = lanes(in_mask(mb) && hit != 0u);
                if (!mm) break;
                uint32_t sg = 0;
                if (hit) {
                    const uint32_t k = (uint32_t)__builtin_ctz(hit);
                    hit &= hit - 1u;
                    sg = (uint32_t)c * seg_cap + seg_cap - 1u - (base + k);
                }
                stream8(mm, sg);
            }
            base += 16;
            mb &= lanes(base < nb);
            if (!mb) break;
            if (in_mask(mb)) {  // directory bytes past the header's 16 (a skewed chunk)
                const u32x4 q = *reinterpret_cast<const u32x4*>(dir + c * (int64_t)dir_cap + base);
                const uint32_t e[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    hit |= (((e[k >> 2] >> (8 * (k & 3))) & 0xFFu) == bb && base + k < nb) ? 1u << k : 0u;
            }
        }
    }
    __syncthreads();
    uint32_t* out = part_ch + (int64_t)blockIdx.x * hn;
    for (int i = threadIdx.x; i < hn; i += kCRT) out[i] = h[slot(i)];
}

// ---- pair reduce --------------------------------------------------------------------
// A pair (a, b), b >= a, of a bucket is counted in one of two LDS structures:
//   band   dense counters band[a_local * D + (b - a)] for b - a < D = 2^dbits
//   hash   open addressing (key = a_local << bbits | b) for the other pairs.
constexpr int kRT = 1024;               // pair-reduce threads (16 waves)
constexpr int kBand = 8192;             // band counters per bucket (32 KB)
constexpr int kHashR = 4096;            // hash slots per pair-reduce block
constexpr int kHashF = 8192;            // hash slots per final (per-bucket) block
#ifndef KARMA_FINAL_THREADS
#define KARMA_FINAL_THREADS 512  // 1024: 8-rank strong preview 0.151-0.169 against 0.145-0.148 ms (r06t)
#endif
constexpr int kFT = KARMA_FINAL_THREADS;  // final-kernel threads
constexpr int kSlotCap = kBand + kHashF;  // output pairs per bucket, at most

template <int CAP, int THREADS>
struct HTab {
    uint32_t* keys;
    uint32_t* vals;
    int* nuniq;
    __device__ void init() {
        for (int t = threadIdx.x; t < CAP; t += THREADS) {
            keys[t] = kEmpty;
            vals[t] = 0;
        }
        if (threadIdx.x == 0) *nuniq = 0;
    }
    // false when CAP slots were probed without room (callers flag overflow)
    __device__ __forceinline__ bool insert(uint32_t key, uint32_t c) {
        uint32_t h = hash32(key) & (CAP - 1);
        for (int probe = 0; probe < CAP; ++probe) {
            const uint32_t k = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (k == key) {
                atomicAdd(&vals[h], c);
                return true;
            }
            if (k == kEmpty) {
                const uint32_t old = atomicCAS(&keys[h], kEmpty, key);
                if (old == kEmpty || old == key) {
                    if (old == kEmpty) atomicAdd(nuniq, 1);
                    atomicAdd(&vals[h], c);
                    return true;
                }
            }
            h = (h + 1) & (CAP - 1);
        }
        return false;
    }
    // occupied slots to the front; returns their number (all threads)
    __device__ int compact(int* cnt) {
        if (threadIdx.x == 0) *cnt = 0;
        __syncthreads();
        uint32_t my_k[CAP / THREADS], my_v[CAP / THREADS];
#pragma unroll
        for (int u = 0; u < CAP / THREADS; ++u) {
            my_k[u] = keys[u * THREADS + threadIdx.x];
            my_v[u] = vals[u * THREADS + threadIdx.x];
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < CAP / THREADS; ++u) {
            if (my_k[u] != kEmpty) {
                const int pos = atomicAdd(cnt, 1);
                keys[pos] = my_k[u];
                vals[pos] = my_v[u];
            }
        }
        __syncthreads();
        return *cnt;
    }
};

// One block per (pair bucket, group of flushes).  Output: the group's dense
// band counters and its compacted hash list (part_n = -1: no flush in group).
__global__ void __launch_bounds__(kRT) pair_reduce_kernel(const uint32_t* __restrict__ pent, RunDir dir,
                                                          int n_pg, int bw, int bbits, int dbits, int B,
                                                          uint32_t* __restrict__ part_band,
                                                          uint32_t* __restrict__ part_keys,
                                                          uint32_t* __restrict__ part_cnt, int* __restrict__ part_n,
                                                          uint8_t* __restrict__ overflow) {
    __shared__ uint32_t band[kBand];
    __shared__ uint32_t hkeys[kHashR];
    __shared__ uint32_t hvals[kHashR];
    __shared__ int nuniq, cnt, ovf;
    __shared__ int slots[kRT];
    HTab<kHashR, kRT> t{hkeys, hvals, &nuniq};
    const int bucket = blockIdx.x / n_pg, grp = blockIdx.x % n_pg;
    const int band_n = dbits >= 0 ? (1 << (bw + dbits)) : 0;
    const uint32_t D = dbits >= 0 ? (1u << dbits) : 0u;
    int64_t f_lo, f_hi;
    group_range(dir.n, n_pg, grp, &f_lo, &f_hi);
    const int64_t sl = blockIdx.x;
    if (f_lo >= f_hi) {  // no pairs in this group (uniform)
        if (threadIdx.x == 0) part_n[sl] = -1;
        return;
    }
    t.init();
    for (int i = threadIdx.x; i < band_n; i += kRT) band[i] = 0;
    if (threadIdx.x == 0) ovf = 0;
    __syncthreads();
    const uint32_t bmask = (1u << bbits) - 1u, abase = (uint32_t)bucket << bw;
    // a full table (rare) is flagged in LDS: a local flag whose address the
    // stream's stop check takes lived in scratch (a scratch access per pair)
    auto add = [&](uint32_t e) {
        if (e == kEmpty) return;
        const uint32_t al = e >> bbits, d = (e & bmask) - (abase + al);
        if (d < D)
            __hip_atomic_fetch_add(&band[(al << dbits) | d], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else if (!t.insert(e, 1u))
            ovf = 1;
    };
    stream_runs(
        reinterpret_cast<const u32x4*>(pent), f_lo, f_hi, kRT,
        [&](int64_t f, int64_t* beg, uint32_t* len) {
            const uint32_t* o = dir.off + f * (B + 1) + bucket;
            *beg = (dir.base[f] + o[0]) >> 2;
            *len = (o[1] - o[0]) >> 2;
        },
        [&](const u32x4 v) {
            add(v.x), add(v.y), add(v.z), add(v.w);
            if (nuniq > kHashR - kHashR / 8) ovf = 1;  // early out: the bucket goes generic
        },
        &ovf, slots);
    __syncthreads();
    if (ovf) {
        if (threadIdx.x == 0) overflow[bucket] = 1;
        return;
    }
    uint32_t* pb = part_band + sl * (int64_t)kBand;
    for (int i = threadIdx.x; i < band_n; i += kRT) pb[i] = band[i];
    const int n = t.compact(&cnt);
    uint32_t* pk = part_keys + sl * (int64_t)kHashR;
    uint32_t* pc = part_cnt + sl * (int64_t)kHashR;
    for (int i = threadIdx.x; i < n; i += kRT) {
        pk[i] = hkeys[i];
        pc[i] = hvals[i];
    }
    if (threadIdx.x == 0) part_n[sl] = n;
}

// Summed code histogram entry gi = (m0 << 3 | M), m0 a global contig index.
__device__ __forceinline__ uint32_t code_count(const uint32_t* __restrict__ part_ch, int n_cg, int bwc, int gi) {
    const int bc = gi >> (bwc + 3), i = gi & ((8 << bwc) - 1);
    const int hn = 8 << bwc;
    uint32_t k = 0;
    for (int g = 0; g < n_cg; ++g) k += part_ch[((int64_t)bc * n_cg + g) * hn + i];
    return k;
}

// One block per pair bucket: sum the groups' bands, add the compact reads'
// pairs, merge the hash lists, and write the bucket's pairs sorted by (a, b).
// Band pairs and hash pairs are disjoint (b - a < D vs >= D); a pair's output
// position is its rank in its own sorted list plus the number of smaller keys
// in the other one.
// HF hash slots: one group's list (n_pg = 1, < kHashR keys) fits 4096, and the
// block then takes 68 KB of LDS (2 blocks per CU for the many small buckets of
// a large n_contigs); several groups' lists are merged in 8192.
// Owner bounds of an exchange (karma_graph_split_hint): the final kernel of the
// bucket holding bound r writes the number of its keys with a < bounds[r].
constexpr int kMaxSplit = 65;  // 64 ranks
struct SplitArgs {
    int n;
    int64_t b[kMaxSplit];
    int64_t* out;  // per bound: keys of its bucket below it
};

template <int HF>
__global__ void __launch_bounds__(kFT) final_kernel(
    int n_pg, int n_cg, int bw, int bbits, int dbits, int bwc, const uint32_t* __restrict__ part_band,
    const uint32_t* __restrict__ part_ch, const uint32_t* __restrict__ part_keys,
    const uint32_t* __restrict__ part_cnt, const int* __restrict__ part_n, uint64_t* __restrict__ out_keys,
    int64_t* __restrict__ out_counts, int64_t* __restrict__ out_n, uint8_t* __restrict__ overflow, SplitArgs split,
    uint64_t* __restrict__ lb, int64_t* __restrict__ out_off) {
    __shared__ uint32_t bsum[kBand];
    __shared__ uint32_t rowpos[(kBand >> 3) + 1];  // nonzero band slots before row a_local (D = 8 on this path)
    __shared__ uint32_t hkeys[HF];
    __shared__ uint32_t hvals[HF];
    __shared__ uint32_t wsum[kFT / 64];
    __shared__ int nuniq, cnt;
    __shared__ int64_t base;
    const int bucket = blockIdx.x;
    // a bucket on the generic path (overflow) takes no room in the array: the
    // host rebuilds the list from the per-bucket sources (SetsJob::finish)
    auto skip = [&]() {
        if (threadIdx.x < 64) {
            const int64_t o = lookback_offset(lb, bucket, 0, (int)threadIdx.x);
            if (threadIdx.x == 0) {
                out_off[bucket] = o;
                out_n[bucket] = 0;
                if (bucket == (int)gridDim.x - 1) out_off[bucket + 1] = o;
            }
        }
    };
    if (overflow[bucket]) {  // generic path
        skip();
        return;
    }
    HTab<HF, kFT> t{hkeys, hvals, &nuniq};
    const int band_n = dbits >= 0 ? (1 << (bw + dbits)) : 0;
    // one group (HF == kHashR): its list is already unique, copied as is
    constexpr bool one_list = HF == kHashR;
    if (!one_list) t.init();
    for (int i = threadIdx.x; i < band_n; i += kFT) {
        uint32_t v = 0;
        for (int gi = 0; gi < n_pg; ++gi) {
            const int64_t sl = (int64_t)bucket * n_pg + gi;
            if (part_n[sl] >= 0) v += part_band[sl * kBand + i];
        }
        bsum[i] = v;
    }
    __syncthreads();
    // compact reads: a code (m0, M) with count k adds k to every pair
    // (m0 + i, m0 + j), i <= j, of its contigs; this bucket takes the pairs
    // with m0 + i inside it, from codes with m0 in [start - 3, end)
    if (n_cg > 0) {
        // a thread per first contig m0 (its 8 codes M = 0..7 as two 16-byte
        // loads per group, every group's loads in flight together); the codes'
        // pairs are summed in registers, then at most 10 LDS atomics per m0
        // (code M: contigs m0 + i for the set bits i of 1 | M << 1)
        const int hn = 8 << bwc;
        for (int m0l = (bucket > 0 ? -3 : 0) + (int)threadIdx.x; m0l < (1 << bw); m0l += kFT) {
            const int64_t gi = ((int64_t)bucket << (bw + 3)) + 8 * (int64_t)m0l;  // code (m0, 0)
            const uint4* src = reinterpret_cast<const uint4*>(part_ch + (gi >> (bwc + 3)) * n_cg * hn + (gi & (hn - 1)));
            uint32_t k[8] = {};
            for (int g = 0; g < n_cg; ++g) {
                const uint4 a = src[(int64_t)g * (hn >> 2)], b = src[(int64_t)g * (hn >> 2) + 1];
                k[0] += a.x, k[1] += a.y, k[2] += a.z, k[3] += a.w;
                k[4] += b.x, k[5] += b.y, k[6] += b.z, k[7] += b.w;
            }
#pragma unroll
            for (int i1 = 0; i1 < 4; ++i1) {
                if (m0l + i1 < 0 || m0l + i1 >= (1 << bw)) continue;
#pragma unroll
                for (int j1 = i1; j1 < 4; ++j1) {
                    uint32_t acc = 0;
#pragma unroll
                    for (int M = 0; M < 8; ++M) {
                        const uint32_t bits = 1u | (uint32_t)M << 1;
                        if ((bits >> i1 & 1u) && (bits >> j1 & 1u)) acc += k[M];
                    }
                    if (acc) atomicAdd(&bsum[(m0l + i1) << dbits | (j1 - i1)], acc);
                }
            }
        }
        __syncthreads();
    }
    int nh;
    if (one_list) {
        nh = max(0, part_n[bucket]);
        for (int i = threadIdx.x; i < nh; i += kFT) {
            hkeys[i] = part_keys[(int64_t)bucket * kHashR + i];
            hvals[i] = part_cnt[(int64_t)bucket * kHashR + i];
        }
        __syncthreads();
    } else {
        for (int gi = 0; gi < n_pg; ++gi) {
            const int64_t sl = (int64_t)bucket * n_pg + gi;
            const int n = part_n[sl];
            bool full = false;
            for (int i = threadIdx.x; i < n; i += kFT)
                full |= !t.insert(part_keys[sl * kHashR + i], part_cnt[sl * kHashR + i]);
            if (__syncthreads_or(full)) {
                if (threadIdx.x == 0) overflow[bucket] = 1;
                skip();
                return;
            }
        }
        nh = t.compact(&cnt);
    }
    int p2 = 1;
    while (p2 < nh) p2 <<= 1;
    for (int i = nh + threadIdx.x; i < p2; i += kFT) {
        hkeys[i] = kEmpty;
        hvals[i] = 0;
    }
    __syncthreads();
    if (nh > 1) lds_bitonic(hkeys, hvals, p2);
    // band output positions: wave w takes a segment of the band, lane l the
    // slots seg + l + 64k (coalesced stores); a slot's rank among the nonzero
    // slots comes from ballots, the segments' bases from their totals
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int seg_len = max(64, band_n / (kFT / 64));
    const int seg0 = wave * seg_len, seg1 = min(band_n, seg0 + seg_len);
    const unsigned long long lt = (1ull << lane) - 1ull;
    {
        uint32_t nz = 0;
        for (int e0 = seg0; e0 < seg1; e0 += 64) nz += (uint32_t)__popcll(__ballot(bsum[e0 + lane] != 0));
        if (lane == 0) wsum[wave] = nz;
    }
    __syncthreads();
    uint32_t run = 0, nb = 0;
    for (int w = 0; w < kFT / 64; ++w) {
        const uint32_t c = wsum[w];
        run += w < wave ? c : 0u;
        nb += c;
    }
    if (wave == 0) {
        const int64_t o = lookback_offset(lb, bucket, (int64_t)nb + nh, lane);
        if (lane == 0) {
            base = o;
            out_off[bucket] = o;
            if (bucket == (int)gridDim.x - 1) out_off[bucket + 1] = o + nb + nh;  // the list's length
        }
    }
    __syncthreads();
    const uint32_t bmask = (1u << bbits) - 1u;
    const uint64_t abase = (uint64_t)bucket << bw;
    uint64_t* ok = out_keys + base;
    int64_t* oc = out_counts + base;
    for (int e0 = seg0; e0 < seg1; e0 += 64) {
        const int i = e0 + lane;
        const uint32_t c = bsum[i];
        const unsigned long long m = __ballot(c != 0);
        const uint32_t at = run + (uint32_t)__popcll(m & lt);  // nonzero slots before i
        if ((i & ((1 << dbits) - 1)) == 0) rowpos[i >> dbits] = at;
        if (c) {
            const uint32_t al = (uint32_t)i >> dbits, b = (uint32_t)abase + al + ((uint32_t)i & ((1u << dbits) - 1u));
            const uint32_t key = (al << bbits) | b;
            int lo = 0, hi = nh;  // hash keys below key
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (hkeys[mid] < key) lo = mid + 1;
                else hi = mid;
            }
            ok[at + lo] = ((abase + al) << 32) | b;
            oc[at + lo] = c;
        }
        run += (uint32_t)__popcll(m);
    }
    if (threadIdx.x == 0 && band_n) rowpos[band_n >> dbits] = nb;
    __syncthreads();
    for (int j = threadIdx.x; j < nh; j += kFT) {
        const uint32_t k = hkeys[j], al = k >> bbits;
        const uint32_t below = band_n ? rowpos[min((int)(al + 1), band_n >> dbits)] : 0u;
        const uint32_t pos = j + below;
        ok[pos] = ((abase + al) << 32) | (k & bmask);
        oc[pos] = hvals[j];
    }
    if (threadIdx.x == 0) out_n[bucket] = nb + nh;
    if (split.n) {
        // keys of this bucket with a below the bound: the band's nonzero slots
        // in the rows before it (rowpos) plus the hash keys before its row
        // (sorted in LDS), no search over the list just written
        const int64_t c_lo = (int64_t)bucket << bw, c_hi = c_lo + (int64_t(1) << bw);
        for (int r = threadIdx.x; r < split.n; r += kFT) {
            const int64_t bd = split.b[r];
            if (bd < c_lo || bd >= c_hi) continue;
            const uint32_t al = (uint32_t)(bd - c_lo);
            const uint32_t lim = al << bbits;
            int lo = 0, hi = nh;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (hkeys[mid] < lim) lo = mid + 1;
                else hi = mid;
            }
            split.out[r] = (int64_t)(band_n ? rowpos[al] : 0u) + lo;
        }
    }
}

// ---- overflow fallback: every pair of one bucket as (key, count), generic sort ----
// Thread t handles pair-stream flush t (this bucket's run) and compact-read
// code t of the bucket (codes with m0 in [start - 3, end)).
__global__ void bucket_widen_kernel(const uint32_t* __restrict__ pent, RunDir dir, int B, int bucket, int bw,
                                    int bbits, const uint32_t* __restrict__ part_ch, int n_cg, int bwc,
                                    uint64_t* __restrict__ out_k, int64_t* __restrict__ out_c,
                                    unsigned long long* __restrict__ n_out, int count_only) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t abase = (uint64_t)bucket << bw;
    const int64_t n_fl = *dir.n;
    unsigned long long n = 0, at = 0;
    for (int pass = count_only ? 1 : 0; pass < 2; ++pass) {
        // pass 0 counts this thread's pairs, pass 1 emits (or only counts)
        auto emit = [&](uint64_t key, int64_t c) {
            if (pass == 0 || count_only) {
                ++n;
            } else {
                out_k[at] = key;
                out_c[at] = c;
                ++at;
            }
        };
        if (pass == 1 && !count_only) {
            if (!n) return;
            at = atomicAdd(n_out, n);
        }
        if (t < n_fl) {  // pair entries of flush t
            const uint32_t* o = dir.off + t * (B + 1) + bucket;
            const int64_t beg = dir.base[t] + o[0];
            for (uint32_t i = 0; i < o[1] - o[0]; ++i) {
                const uint32_t k = pent[beg + i];
                if (k != kEmpty) emit(((abase + (k >> bbits)) << 32) | (k & ((1u << bbits) - 1u)), 1);
            }
        }
        const int64_t ci = t - (bucket > 0 ? 24 : 0);  // code index relative to the bucket start
        if (n_cg > 0 && t < (8 << bw) + (bucket > 0 ? 24 : 0)) {
            const uint32_t k = code_count(part_ch, n_cg, bwc, (int)((int64_t)(bucket << (bw + 3)) + ci));
            if (k) {
                const int64_t m0 = (int64_t)abase + (ci >> 3);
                const uint32_t bits = 1u | ((uint32_t)ci & 7u) << 1;
                for (int i1 = 0; i1 < 4; ++i1)
                    for (int j1 = i1; j1 < 4; ++j1)
                        if ((bits >> i1 & 1u) && (bits >> j1 & 1u) && m0 + i1 >= (int64_t)abase &&
                            m0 + i1 < (int64_t)abase + (1 << bw))
                            emit(((uint64_t)(m0 + i1) << 32) | (uint64_t)(m0 + j1), k);
            }
        }
    }
    if (count_only && n) atomicAdd(n_out, n);
}

// big reads (> 8 records): pair keys, one thread per read, O(m^3) dedup
// (count pass: n_out[1] = 1 when a record's contig is >= N; the binned
// flagged classify checks the range of codes only)
__global__ void big_pairs_kernel(RecIn rec, int64_t A, const int64_t* __restrict__ big_list,
                                 int64_t n_big, uint32_t N, uint64_t* __restrict__ out,
                                 unsigned long long* __restrict__ n_out, int count_only,
                                 const uint32_t* __restrict__ remap) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_big) return;
    if (count_only) {
        const int64_t i = big_list[k];
        int64_t e = i;
        bool bad = false;
        do bad |= rec.contig(e) >= N;
        while (++e < A && rec.cont(e));
        if (bad) n_out[1] = 1;
    }
    unsigned long long c = 0;
    auto map = [&](uint32_t x) { return remap && x < N ? remap[x] : x; };
    read_pairs_slow(rec, A, big_list[k], map, [&](uint32_t a, uint32_t b) {
        if (b >= N) return;
        if (count_only) ++c;
        else out[atomicAdd(n_out, 1ull)] = ((uint64_t)a << 32) | b;
    });
    if (count_only && c) atomicAdd(n_out, c);
}

__global__ void fill_ones_i64_kernel(int64_t* __restrict__ v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = 1;
}

// Bucket b's sorted list lies at base + src_off[b] (final_kernel's array), or,
// for a bucket that overflowed the LDS tables, at the generic path's arrays
// (src_k[b] / src_c[b] non-null).  Only after an overflow: otherwise the final
// kernel's array is the list.
__global__ void assemble2_kernel(const uint64_t* __restrict__ base_k, const int64_t* __restrict__ base_c,
                                 const int64_t* __restrict__ src_off, const uint64_t* const* __restrict__ src_k,
                                 const int64_t* const* __restrict__ src_c, const int64_t* __restrict__ n_per,
                                 const int64_t* __restrict__ dst_off, uint64_t* __restrict__ keys,
                                 int64_t* __restrict__ counts) {
    const int64_t b = blockIdx.x;
    const int64_t n = n_per[b], d = dst_off[b];
    const uint64_t* sk = src_k && src_k[b] ? src_k[b] : base_k + src_off[b];
    const int64_t* sc = src_c && src_c[b] ? src_c[b] : base_c + src_off[b];
    for (int64_t t = threadIdx.x; t < n; t += blockDim.x) {
        keys[d + t] = sk[t];
        counts[d + t] = sc[t];
    }
}

int grid_n(int64_t n, int block = 256) { return (int)std::max<int64_t>(1, ceil_div(n, block)); }



}  // namespace

namespace karma {

// The sorted unique list (mk, mc, U) plus the pairs of reads with > 8 records
// (big_list) -> out.
int finish_pairs(karma_ctx* ctx, RecIn rec, int64_t A, int64_t N, const int64_t* big_list, unsigned n_big,
                 DevArray<uint64_t>& mk, DevArray<int64_t>& mc, int64_t U, karma_pairs* out,
                 const uint32_t* remap = nullptr) {
    out->n_contigs = N;
    if (n_big == 0) {
        // no synchronisation: later work on this stream is ordered after the
        // assemble kernel, host reads synchronise, and the records were last
        // read before the control-block read
        out->keys.swap(mk);
        out->counts.swap(mc);
        out->n = U;
        return KARMA_OK;
    }
    DevArray<unsigned long long> np;
    KARMA_TRY(np.alloc(ctx, 2));
    KARMA_HIP(hipMemsetAsync(np.ptr, 0, 16, ctx->stream));
    KARMA_LAUNCH(ctx, "graph_big_count", big_pairs_kernel, grid_n(n_big, 64), 64, 0, rec, A, big_list,
                 (int64_t)n_big, (uint32_t)N, (uint64_t*)nullptr, np.ptr, 1, remap);
    unsigned long long hpb[2] = {0, 0};
    KARMA_HIP(hipMemcpyAsync(hpb, np.ptr, 16, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    const unsigned long long hp = hpb[0];
    KARMA_CHECK(!hpb[1], KARMA_ERR_ARG, "a record's contig index is >= n_contigs (%lld)", (long long)N);
    DevArray<uint64_t> allk;
    DevArray<int64_t> allc;
    KARMA_TRY(allk.alloc(ctx, U + hp));
    KARMA_TRY(allc.alloc(ctx, U + hp));
    if (U) {
        KARMA_HIP(hipMemcpyAsync(allk.ptr, mk.ptr, U * 8, hipMemcpyDeviceToDevice, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(allc.ptr, mc.ptr, U * 8, hipMemcpyDeviceToDevice, ctx->stream));
    }
    KARMA_HIP(hipMemsetAsync(np.ptr, 0, 8, ctx->stream));
    KARMA_LAUNCH(ctx, "graph_big_pairs", big_pairs_kernel, grid_n(n_big, 64), 64, 0, rec, A, big_list,
                 (int64_t)n_big, (uint32_t)N, allk.ptr + U, np.ptr, 0, remap);
    KARMA_LAUNCH(ctx, "fill_ones", fill_ones_i64_kernel, grid_n(hp), 256, 0, allc.ptr + U, (int64_t)hp);
    KARMA_TRY(sort_reduce_pairs(ctx, allk.ptr, allc.ptr, nullptr, U + (int64_t)hp, 64, out->keys, out->counts,
                                nullptr, &out->n));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    return KARMA_OK;
}

// per-chunk pair lists -> one contiguous list of ones-counted keys
__global__ void widen_counts_kernel(const uint32_t* __restrict__ n, int64_t m, int64_t* __restrict__ w) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= m) w[i] = i < m ? (int64_t)n[i] : 0;
}

__global__ void gather_lists_kernel(const uint64_t* __restrict__ lists, int64_t cap, const uint32_t* __restrict__ n,
                                    const int64_t* __restrict__ off, uint64_t* __restrict__ keys,
                                    int64_t* __restrict__ ones) {
    const int64_t c = blockIdx.x;
    const uint64_t* src = lists + c * cap;
    const int64_t d = off[c];
    for (uint32_t t = threadIdx.x; t < n[c]; t += blockDim.x) {
        keys[d + t] = src[t];
        ones[d + t] = 1;
    }
}

// n_contigs > 2^21: bucket-local 32-bit pair keys (a_local << bbits | b) no
// longer fit, so every read takes the general path (sorted distinct contigs,
// per-chunk u64 pair lists, no atomics) and one 64-bit sort-reduce follows;
// reads of > 8 records are merged as in the main path.
int records_to_pairs_wide(karma_ctx* ctx, RecIn rec, int64_t A, int64_t N, karma_pairs* out) {
    KARMA_CHECK(N >= 1 && N <= (int64_t(1) << 24), KARMA_ERR_ARG, "n_contigs %lld out of range [1, 2^24]",
                (long long)N);
    int bbits = 1;
    while ((int64_t(1) << bbits) < N) ++bbits;
    const int64_t n_chunks = std::max<int64_t>(1, ceil_div(A, kCChunk));
    DevArray<uint32_t> codes, n_codes, n_gen, n_pl;
    DevArray<int64_t> big_list, ctrl, widths, off;
    DevArray<unsigned long long> blk_items;
    KARMA_TRY(codes.alloc(ctx, n_chunks * kCChunk));
    KARMA_TRY(n_codes.alloc(ctx, n_chunks));
    KARMA_TRY(n_gen.alloc(ctx, n_chunks));
    KARMA_TRY(n_pl.alloc(ctx, n_chunks));
    KARMA_TRY(big_list.alloc(ctx, A / (kMaxFast + 1) + 1));
    KARMA_TRY(blk_items.alloc(ctx, 2 * n_chunks));
    KARMA_TRY(widths.alloc(ctx, n_chunks + 1));
    KARMA_TRY(off.alloc(ctx, n_chunks + 1));
    KARMA_TRY(ctrl.alloc(ctx, 4));  // flags[4] | counters[3] (big reads) | spare
    int* const flags = reinterpret_cast<int*>(ctrl.ptr);
    unsigned* const counters = reinterpret_cast<unsigned*>(ctrl.ptr + 2);
    void* hpin = nullptr;
    KARMA_TRY(ctx_pinned(ctx, 5 * 8, &hpin));
    int64_t* const h = static_cast<int64_t*>(hpin);
    int64_t pcap = kCChunk / 8;
    DevArray<uint64_t> plist;
    int64_t P = 0;
    unsigned n_big = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        KARMA_TRY(plist.alloc(ctx, n_chunks * pcap));
        KARMA_HIP(hipMemsetAsync(ctrl.ptr, 0, 4 * 8, ctx->stream));
        KARMA_HIP(hipMemsetAsync(blk_items.ptr, 0, 2 * n_chunks * 8, ctx->stream));
        KARMA_HIP(hipMemsetAsync(n_gen.ptr, 0, n_chunks * 4, ctx->stream));
        if (A > 0) {
            ClassArgs C{rec.pr,    A,         (uint32_t)N, false,         codes.ptr, n_codes.ptr,
                        n_gen.ptr, blk_items.ptr, 1,     big_list.ptr, counters,  flags,
                        nullptr,   0,         0,       nullptr, 0, nullptr, kCChunk};
            C.recw = rec.fw;
            if (rec.flagged())
                KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<false, false, false, false, true>),
                             ceil_div(n_chunks, kCW / 64), kCW, 0, C, BinArgs{});
            else
                KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<false, false>), ceil_div(n_chunks, kCW / 64), kCW,
                             0, C, BinArgs{});
        }
        KARMA_LAUNCH(ctx, "graph_general", general_kernel, general_grid(ctx, n_chunks), kGW, 0, rec, A, (uint32_t)N,
                     codes.ptr, n_gen.ptr, n_chunks, plist.ptr, pcap, n_pl.ptr, blk_items.ptr + n_chunks, 1, flags,
                     (const uint32_t*)nullptr, (const unsigned*)nullptr, kCChunk);
        KARMA_LAUNCH(ctx, "widen_counts", widen_counts_kernel, grid_n(n_chunks + 1), 256, 0, n_pl.ptr, n_chunks,
                     widths.ptr);
        KARMA_TRY(scan_excl_i64(ctx, widths.ptr, off.ptr, n_chunks + 1));
        KARMA_HIP(hipMemcpyAsync(h, ctrl.ptr, 4 * 8, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(h + 4, off.ptr + n_chunks, 8, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
        const int* hf = reinterpret_cast<const int*>(h);
        KARMA_CHECK(!hf[0], KARMA_ERR_UNSORTED, "records are not grouped by read (read ids decrease)");
        KARMA_CHECK(!hf[1], KARMA_ERR_ARG, "a record's contig index is >= n_contigs (%lld)", (long long)N);
        n_big = reinterpret_cast<const unsigned*>(h + 2)[0];
        P = h[4];
        if (!hf[2]) break;
        KARMA_CHECK(attempt == 0, KARMA_ERR_STATE, "pair list capacity exceeded twice");
        pcap = kCChunk * 9 / 2;  // every read with <= 8 records fits
    }
    DevArray<uint64_t> keys;
    DevArray<int64_t> ones;
    KARMA_TRY(keys.alloc(ctx, P));
    KARMA_TRY(ones.alloc(ctx, P));
    if (P) KARMA_LAUNCH(ctx, "gather_lists", gather_lists_kernel, n_chunks, 256, 0, plist.ptr, pcap, n_pl.ptr,
                        off.ptr, keys.ptr, ones.ptr);
    DevArray<uint64_t> mk;
    DevArray<int64_t> mc;
    int64_t U = 0;
    KARMA_TRY(sort_reduce_pairs(ctx, keys.ptr, ones.ptr, nullptr, P, 32 + bbits, mk, mc, nullptr, &U));
    return finish_pairs(ctx, rec, A, N, big_list.ptr, n_big, mk, mc, U, out);
}

// ---- relabelling for contig orders without locality ---------------------------
// The compact path needs the contigs of a read within 4 ids.  When the FASTA
// order does not list isoforms together, most reads take the general path
// (8.7 ms instead of 1.3 at config 3).  relabel_probe_kernel then asks for one
// relabelled rerun (> 1/8 of the probed reads span more than 4 ids; classify
// and the general kernel skip this pass): each contig is hooked to the smallest
// contig it shares a
// read with, the hooks are followed to a root, and contigs are renumbered
// root by root, so contigs that share reads get adjacent ids.  The pipeline
// reruns on the new ids (read through the remap table as records are read) and
// the resulting pair keys are mapped back and re-sorted: the output is the
// same; only the reads' path changes.
// The decision, before classify: kRelabelProbes reads at evenly spaced
// record positions (the next read start at or after each), non-compact when
// their distinct contigs span more than 4 ids.  One block, one round of loads.
constexpr int kRelabelProbes = 256;

__global__ void __launch_bounds__(kRelabelProbes) relabel_probe_kernel(RecIn rec, int64_t A,
                                                                       uint32_t N, unsigned* __restrict__ relabel,
                                                                       uint64_t* __restrict__ zero, int64_t n_zero) {
    __shared__ unsigned wide;
    // the job's control block (flags, counters, per-bucket sizes; relabel is
    // one of its words) is cleared here: no memset launch ahead of the probe.
    // Thread 0 clears the word holding the relabel flag and sets the flag, so
    // the barriers order LDS only (no wait for the clearing stores)
    const int64_t rw = (int64_t)(reinterpret_cast<uintptr_t>(relabel) - reinterpret_cast<uintptr_t>(zero)) / 8;
    if (threadIdx.x == 0) {
        wide = 0;
        if (rw >= 0 && rw < n_zero) zero[rw] = 0;
    }
    for (int64_t i = threadIdx.x; i < n_zero; i += kRelabelProbes)
        if (i != rw) zero[i] = 0;
    lds_barrier();
    // a window of 32 records from an even position, loaded at once (16 B each)
    constexpr int kW = 32;
    const int64_t p = (A * (int64_t)threadIdx.x / kRelabelProbes) & ~int64_t(1);
    uint32_t rid[kW], ctg[kW];
    if (p + kW <= A) {
        if (rec.flagged()) {  // rid[j]: the raw word (bit 31 starts a read)
#pragma unroll
            for (int j = 0; j < kW; ++j) rid[j] = rec.fw[p + j], ctg[j] = rid[j] & kContigMask;
        } else {
            const u32x4* v = reinterpret_cast<const u32x4*>(rec.pr + p);
#pragma unroll
            for (int u = 0; u < kW / 2; ++u) {
                const u32x4 q = v[u];
                rid[2 * u] = q.x, ctg[2 * u] = q.y, rid[2 * u + 1] = q.z, ctg[2 * u + 1] = q.w;
            }
        }
        // the first read that starts inside the window and ends inside it
        int s0 = -1, e0 = -1;
#pragma unroll
        for (int j = 1; j < kW; ++j) {
            const bool start = rec.flagged() ? (int)rid[j] < 0 : rid[j] != rid[j - 1];
            if (start && s0 >= 0 && e0 < 0) e0 = j;
            if (start && s0 < 0) s0 = j;
        }
        if (s0 > 0 && e0 > 0) {
            uint32_t mn = kEmpty, mx = 0;
#pragma unroll
            for (int j = 0; j < kW; ++j)
                if (j >= s0 && j < e0) mn = min(mn, ctg[j]), mx = max(mx, ctg[j]);
            if (mx - mn > 3u && mx < N) atomicAdd(&wide, 1u);
        }
    }
    lds_barrier();
    if (threadIdx.x == 0 && wide * 8 > kRelabelProbes) *relabel = 1;
}

__global__ void iota_u32_kernel(uint32_t* __restrict__ v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

// one thread per record; the thread at a read's first record hooks each of the
// read's contigs to the read's smallest contig (test before the atomic)
__global__ void relabel_hook_kernel(RecIn rec, int64_t A, uint32_t N, uint32_t* __restrict__ rep) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A) return;
    if (i > 0 && rec.cont(i)) return;
    uint32_t m = kEmpty;
    int64_t e = i;
    do {
        const uint32_t y = rec.contig(e);
        if (y < N) m = min(m, y);
        ++e;
    } while (e < A && rec.cont(e));
    if (m == kEmpty) return;
    for (int64_t j = i; j < e; ++j) {
        const uint32_t c = rec.contig(j);
        if (c < N && rep[c] > m) atomicMin(&rep[c], m);
    }
}

// root of each contig (hooks only point to smaller ids), and the roots' sizes
__global__ void relabel_root_kernel(const uint32_t* __restrict__ rep, uint32_t N, uint32_t* __restrict__ root,
                                    int64_t* __restrict__ size) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c > N) return;
    if (c == N) {
        size[N] = 0;
        return;
    }
    uint32_t r = (uint32_t)c;
    while (rep[r] != r) r = rep[r];
    root[c] = r;
    atomicAdd(reinterpret_cast<unsigned long long*>(size + r), 1ull);
}

// new id = the root's base + a slot in its group (order inside a group is free)
__global__ void relabel_assign_kernel(const uint32_t* __restrict__ root, const int64_t* __restrict__ base, uint32_t N,
                                      unsigned* __restrict__ fill, uint32_t* __restrict__ remap,
                                      uint32_t* __restrict__ inv) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= N) return;
    const uint32_t r = root[c];
    const uint32_t id = (uint32_t)base[r] + atomicAdd(&fill[r], 1u);
    remap[c] = id;
    inv[id] = (uint32_t)c;
}

// pair keys (a << 32 | b) in new ids -> original ids, a <= b again
__global__ void relabel_back_kernel(uint64_t* __restrict__ keys, int64_t n, const uint32_t* __restrict__ inv) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    const uint32_t a = inv[(uint32_t)(k >> 32)], b = inv[(uint32_t)k];
    keys[i] = (uint64_t)min(a, b) << 32 | max(a, b);
}

// Records (grouped by read, 16-byte aligned) -> sorted unique (a<<32|b, count).
// One compact-path graph call, split at its only common-path synchronisation:
// begin() sizes the scratch and enqueues classify .. final plus the control
// block readback; end() waits, checks, reruns on a full pair list, and
// assembles.  Between the two the host may enqueue unrelated work (the k-mer
// profile on a side stream).
#ifndef KARMA_MARK_AT
#define KARMA_MARK_AT 5
#endif
// where side-stream work (the k-mer profile) may start, see SetsJob::launch;
// KARMA_MARK_AT in the environment overrides the default (scheduling only:
// every position runs the same kernels)
// the general-read branch on the context's fork stream beside the code branch
// (KARMA_FORK=0 in the environment: both branches in order on one stream;
// scheduling only, the same kernels run)
// the binned classify where it applies (KARMA_BIN=0 in the environment: the
// code partition instead, A/B and tests; read per job)
bool bin_on() {
    const char* e = std::getenv("KARMA_BIN");
    return e ? std::atoi(e) != 0 : true;
}
// the code reduce's LDS list of chunks with back segments (KARMA_BACKLIST in
// the environment lowers it, so tests reach the overflow path; read per job)
uint32_t back_list_cap() {
    const char* e = std::getenv("KARMA_BACKLIST");
    const int v = e ? std::atoi(e) : kBackList;
    return (uint32_t)std::max(0, std::min(v, kBackList));
}
bool fork_on() {
    static const bool on = [] {
        const char* e = std::getenv("KARMA_FORK");
        return e ? std::atoi(e) != 0 : true;
    }();
    return on;
}
// Records per classify chunk (one wave each, 4 waves per SIMD resident).  A
// launch of few chunks per wave slot ends in a partial round: 38.6M records
// (config 3 over 8 ranks) are 4,711 chunks of 8192 on 4,096 slots.  Half-size
// chunks while 8192-record chunks would fill fewer than 4 rounds: classify
// 0.0755 -> 0.070 ms there, 0.139 -> 0.128 ms at 4 ranks; at config 3 on one
// GPU (9.2 rounds) 8192 stays, 4096 measured 0.536 -> 0.549 ms
// (profiles/r03/measurements.md (ab_chunk)).
// KARMA_CHUNK=4096|8192 in the environment pins the size (tests run both
// sizes on the same small inputs; read per call).
int64_t chunk_records(const karma_ctx* ctx, int64_t A) {
    if (const char* e = std::getenv("KARMA_CHUNK")) {
        const int64_t c = std::atoll(e);
        if (c == kCChunk || c == kCChunk / 2 || c == kCChunk / 4) return c;
    }
    const int64_t slots = (int64_t)ctx->cu_count * 16;
    return ceil_div(A, kCChunk) < 4 * slots ? kCChunk / 2 : kCChunk;
}
// KARMA_MARK_AT in the environment wins; else the caller's choice
// (ctx->mark_pos, the native step's deferred batches), else the default
int mark_at(const karma_ctx* ctx) {
    static const int env = [] {
        const char* e = std::getenv("KARMA_MARK_AT");
        return e ? std::atoi(e) : -1;
    }();
    return env >= 0 ? env : ctx->mark_pos >= 0 ? ctx->mark_pos : KARMA_MARK_AT;
}
struct SetsJob {
    karma_ctx* ctx = nullptr;
    RecIn rec;
    int64_t A = 0, N = 0;
    Geo g{};
    int B = 0;
    int64_t n_chunks = 0;
    int64_t chunk = kCChunk;  // records per classify chunk (chunk_records)
    bool wide_c = false, wide_p = false, append = false;
    int lpb = 0;
    int64_t n_pblk = 0;
    DevArray<uint32_t> codes, n_codes, n_gen, n_pl;
    DevArray<int64_t> big_list;
    // control block, cleared by one memset and read back by one copy:
    // flags[4] | counters[3] (big reads, code flushes, pair flushes) | spare[2]
    // | pairs per bucket[B+1] | their exclusive scan[B+1] | overflow[B]
    int64_t ctrl_words = 0;
    DevArray<int64_t> ctrl;
    int64_t* cb = nullptr;  // the control block: ctrl, or the caller's zeroed one (ext)
    bool ext = false;
    std::vector<int64_t> split_b;  // owner bounds (karma_graph_split_hint), found by the final kernel
    int64_t* split_loc = nullptr;   // in the control block: per bound, keys of its bucket below it
    int* flags = nullptr;
    unsigned* counters = nullptr;
    int64_t* n_per = nullptr;
    uint64_t* lb = nullptr;  // the final kernel's look-back words (zeroed with the control block)
    int64_t* dst = nullptr;
    uint8_t* ovf = nullptr;
    const int64_t* hctrl = nullptr;  // pinned copy of the control block
    int64_t max_cflush = 0, ccap = 0;
    // binned classify (Bc <= kBinMaxBc, not append): segments, headers, back directories
    bool bin = false;
    uint32_t seg_cap = 0;
    int dir_cap = 0;
    bool slotted = false;  // binned fronts as whole 128-byte slots (classify2_kernel's end)
    DevArray<uint16_t> bsegs;
    DevArray<uint32_t> bhdr;  // kBinHdr uint4 per chunk
    DevArray<uint8_t> bdir;
    DevArray<uint16_t> cent;
    DevArray<int64_t> cf_base;
    DevArray<uint32_t> cf_off;
    unsigned long long* blk_items = nullptr;  // per partition block: codes, pairs (after the control block)
    DevArray<uint32_t> blk_hist;             // per partition block: codes per code bucket (append)
    int64_t pcap = kCChunk / 8;
    DevArray<uint64_t> plist;
    DevArray<uint32_t> pent, pf_off;
    DevArray<int64_t> pf_base;
    int n_cg = 0, n_pg = 0;
    int64_t nsl = 0;
    DevArray<uint32_t> part_ch, part_b, part_k, part_c;
    DevArray<int> part_n;
    DevArray<uint64_t> slot_k;
    DevArray<int64_t> slot_c;
    RunDir pdir{};
    int attempt = 0;
    bool deferred = false;                  // no control-block readback (sets_begin_deferred)
    bool relabeled = false;                 // a relabelled rerun (see relabel_probe_kernel)
    DevArray<uint32_t> remap_map, remap_inv;  // new id by old id, old id by new id

    int setup();
    int launch();
    int relabel();
    int finish(karma_pairs* out);
};

int SetsJob::setup() {
    KARMA_TRY(make_geo(N, &g));
    B = g.B;
    chunk = chunk_records(ctx, A);
    n_chunks = std::max<int64_t>(1, ceil_div(A, chunk));
    // partition: one round of resident blocks, each taking consecutive chunk lists
    wide_c = g.Bc > kNarrowBc;
    wide_p = B > kNarrowB;
    // code partition: per-flush padded runs while a flush's runs are long (few
    // code buckets); one appended run per (block, bucket) beyond that
    append = g.Bc >= KARMA_APPEND_MIN_BC;
    const void* code_part = append ? (wide_c ? reinterpret_cast<const void*>(&code_append_kernel<kMaxBc>)
                                             : reinterpret_cast<const void*>(&code_append_kernel<kNarrowBc>))
                                   : (wide_c ? reinterpret_cast<const void*>(&partition_kernel<CodeStreamWide>)
                                             : reinterpret_cast<const void*>(&partition_kernel<CodeStream>));
    const int resident = resident_grid(ctx, code_part, kPT, 0, int64_t(1) << 30);
    lpb = (int)std::min<int64_t>(kMaxListsPerBlock, ceil_div(n_chunks, resident));
    n_pblk = ceil_div(n_chunks, lpb);
    KARMA_TRY(codes.alloc(ctx, n_chunks * chunk));
    KARMA_TRY(n_codes.alloc(ctx, n_chunks));
    KARMA_TRY(n_gen.alloc(ctx, n_chunks));
    KARMA_TRY(n_pl.alloc(ctx, n_chunks));
    KARMA_TRY(big_list.alloc(ctx, A / (kMaxFast + 1) + 1));
    pcap = chunk / 8;
    ctrl_words = 6 + 2 * (int64_t)(B + 1) + ceil_div(B, 8) + (int64_t)split_b.size();
    // one allocation (and one memset per attempt) for the control block and
    // the per-partition-block item counts behind it
    const int64_t cw_total = ctrl_words + 2 * n_pblk + B;
    // a deferred job may take the caller's zeroed block (ctx->job_ctrl)
    ext = deferred && ctx->job_ctrl && ctx->job_ctrl_words >= cw_total;
    static const bool debug_ctrl = std::getenv("KARMA_DEBUG_CTRL") != nullptr;
    if (debug_ctrl)
        std::fprintf(stderr, "[karma] records job: deferred %d, caller block %p (%lld words), needs %lld: %s\n",
                     (int)deferred, (void*)ctx->job_ctrl, (long long)ctx->job_ctrl_words, (long long)cw_total,
                     ext ? "caller's" : "own");
    if (ext) {
        cb = ctx->job_ctrl;
    } else {
        KARMA_TRY(ctrl.alloc(ctx, cw_total));
        cb = ctrl.ptr;
    }
    blk_items = reinterpret_cast<unsigned long long*>(cb + ctrl_words);
    lb = reinterpret_cast<uint64_t*>(cb + ctrl_words + 2 * n_pblk);
    flags = reinterpret_cast<int*>(cb);
    counters = reinterpret_cast<unsigned*>(cb + 2);
    n_per = cb + 6;
    dst = n_per + (B + 1);
    ovf = reinterpret_cast<uint8_t*>(dst + (B + 1));
    split_loc = dst + (B + 1) + ceil_div(B, 8);
    if (!deferred) {
        void* hpin = nullptr;
        KARMA_TRY(ctx_job_pinned(ctx, ctrl_words * 8, &hpin));
        hctrl = static_cast<const int64_t*>(hpin);
    }
    // code stream: <= one code per record + < 8 padding codes per run; a block
    // flushes only a full buffer, and once at its end
    max_cflush = n_pblk + ceil_div(A, CodeStream::kCap) + 1;
    ccap = A + max_cflush * (8 * (int64_t)g.Bc + 8);
    if (append) KARMA_TRY(blk_hist.alloc(ctx, n_pblk * g.Bc));
    // the binned classify (no code partition) while the code buckets' queues
    // fit its LDS; KARMA_BIN=0 in the environment keeps the partition (A/B)
    bin = !append && g.Bc > 0 && g.Bc <= kBinMaxBc && bin_on();
    if (bin) {
        dir_cap = (int)(chunk / kBinQ);
        seg_cap = (uint32_t)(dir_cap + g.Bc);
        // whole slots when a bucket's queue fills well: ~chunk / 3 codes per
        // chunk (3 records per read) over Bc buckets, >= 40 of 64 (config 3:
        // 54; the 8-rank preview's 4,096-record chunks: 27, packed granules)
#ifndef KARMA_BIN_SLOT_MIN
#define KARMA_BIN_SLOT_MIN 120  // records per chunk per bucket for whole slots (0: never)
#endif
        slotted = KARMA_BIN_SLOT_MIN > 0 && A > 0 && chunk >= (int64_t)KARMA_BIN_SLOT_MIN * g.Bc;
        KARMA_CHECK(n_chunks * (int64_t)seg_cap < (int64_t(1) << 32), KARMA_ERR_ARG,
                    "binned classify: %lld chunks exceed 32-bit segment indices", (long long)n_chunks);
        KARMA_TRY(bsegs.alloc(ctx, n_chunks * (int64_t)seg_cap * kBinQ));
        KARMA_TRY(bhdr.alloc(ctx, n_chunks * 4 * kBinHdr));
        KARMA_TRY(bdir.alloc(ctx, n_chunks * (int64_t)dir_cap));
    } else if (g.Bc > 0) {
        KARMA_TRY(cent.alloc(ctx, ccap + 16));
        KARMA_TRY(cf_base.alloc(ctx, max_cflush));
        KARMA_TRY(cf_off.alloc(ctx, max_cflush * (g.Bc + 1)));
    }
    // reduce geometry: grids fixed here, flush ranges from device counters
    // code reduce: one round (one 128 KB-LDS block per CU), at most ~4 flushes per group
    // Groups also cost a 128 KB histogram clear and write-back each (and the
    // final kernel sums them), so a bucket gets one group per ~256K records it
    // may hold (8-way strong scaling of config 3: 3 groups; one group took
    // 0.076 ms against 0.047 for five).
    n_cg = g.Bc > 0 ? (int)std::max<int64_t>(1, std::min<int64_t>({ctx->cu_count / g.Bc, ceil_div(max_cflush, 4),
                                                                     ceil_div(A, (int64_t)g.Bc << KARMA_CG_SHIFT)}))
                    : 0;
    // binned: one group per ~64 chunks at most (a wave's batch), up to one block
    // per CU, and one per 2^19 records a bucket may hold (each group clears and
    // writes back a 128 KB histogram the final kernel sums: at the 8-rank
    // strong preview's 38.6M records 2 groups per bucket instead of 5 took
    // 0.183-0.184 against 0.190-0.192 ms per step; 1: 0.185, 3: 0.188)
    if (bin)
        n_cg = (int)std::max<int64_t>(1, std::min<int64_t>({ctx->cu_count / g.Bc, ceil_div(n_chunks, 64),
                                                            ceil_div(A, (int64_t)g.Bc << 19)}));
    // pair-reduce groups per bucket: enough blocks to fill the chip while
    // buckets are few; one group from KARMA_ONE_GROUP_B buckets on, so the
    // final kernel copies the bucket's single list instead of re-hashing
    n_pg = B >= KARMA_ONE_GROUP_B ? 1 : (int)std::max<int64_t>(1, ceil_div(256, B));
    nsl = (int64_t)B * n_pg;
    if (n_cg) KARMA_TRY(part_ch.alloc(ctx, (int64_t)g.Bc * n_cg * (int64_t(8) << g.bwc)));
    KARMA_TRY(part_b.alloc(ctx, nsl * (int64_t)kBand));
    KARMA_TRY(part_k.alloc(ctx, nsl * (int64_t)kHashR));
    KARMA_TRY(part_c.alloc(ctx, nsl * (int64_t)kHashR));
    KARMA_TRY(part_n.alloc(ctx, nsl));
    KARMA_TRY(slot_k.alloc(ctx, (int64_t)B * kSlotCap));
    KARMA_TRY(slot_c.alloc(ctx, (int64_t)B * kSlotCap));
    return KARMA_OK;
}

// One attempt: every kernel up to the control block readback (no host wait).
int SetsJob::launch() {
    // pair lists: general reads' pairs per chunk; room for 1/8 pair per record
    // first, the bound (4.5 per record) on a rerun
    const int64_t max_pflush = n_pblk + ceil_div(n_chunks * pcap, PairStream::kCap) + 1;
    const int64_t pscap = n_chunks * pcap + max_pflush * (4 * (int64_t)B + 4);
    KARMA_TRY(plist.alloc(ctx, n_chunks * pcap));
    KARMA_TRY(pent.alloc(ctx, pscap + 8));
    KARMA_TRY(pf_base.alloc(ctx, max_pflush));
    KARMA_TRY(pf_off.alloc(ctx, max_pflush * (B + 1)));
    // the probe kernel clears the control block; a caller's block (ext) is zero
    // already on the first attempt, and classify decides the relabel itself
    const bool fresh_ext = ext && attempt == 0 && !relabeled;
    const bool probe = A > 0 && !relabeled && !fresh_ext;
    if (!probe && !fresh_ext) KARMA_HIP(hipMemsetAsync(cb, 0, (ctrl_words + 2 * n_pblk + B) * 8, ctx->stream));
    if (append) KARMA_HIP(hipMemsetAsync(blk_hist.ptr, 0, n_pblk * g.Bc * 4, ctx->stream));
    if (mark_at(ctx) == 3 && attempt == 0 && !relabeled) {  // side-stream work may start beside classify
        if (!ctx->mark_ev) KARMA_HIP(hipEventCreateWithFlags(&ctx->mark_ev, hipEventDisableTiming));
        KARMA_HIP(hipEventRecord(ctx->mark_ev, ctx->stream));
        ctx->mark_set = true;
    }
    if (A > 0) {
        ClassArgs C{rec.pr,    A,         (uint32_t)N,   g.Bc > 0,     codes.ptr, n_codes.ptr,
                    n_gen.ptr, blk_items, lpb, big_list.ptr, counters, flags,
                    append ? blk_hist.ptr : nullptr, g.bwc, g.Bc, relabeled ? remap_map.ptr : nullptr, 0, nullptr,
                    chunk};
        C.recw = rec.fw;
        const BinArgs Bn = bin ? BinArgs{bsegs.ptr, reinterpret_cast<uint4*>(bhdr.ptr), bdir.ptr, (int64_t)seg_cap,
                                         dir_cap, slotted ? 1 : 0}
                               : BinArgs{};
        auto classify = [&](int64_t c_from, int64_t c_to) -> int {
            C.c0 = c_from;
            const int64_t cg = ceil_div(c_to - c_from, kCW / 64);
            if (cg <= 0) return KARMA_OK;
            if (rec.flagged()) {  // flagged records (4 bytes each)
                if (bin && relabeled)
                    KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<false, true, true, true, true>), cg, kCW, 0, C,
                                 Bn);
                else if (bin)
                    KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<false, true, false, true, true>), cg, kCW, 0,
                                 C, Bn);
                else if (append && relabeled)
                    KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<true, true, true, false, true>), cg, kCW, 0,
                                 C, Bn);
                else if (append)
                    KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<true, true, false, false, true>), cg, kCW, 0,
                                 C, Bn);
                else if (relabeled)
                    KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<false, true, true, false, true>), cg, kCW, 0,
                                 C, Bn);
                else
                    KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<false, true, false, false, true>), cg, kCW, 0,
                                 C, Bn);
            } else if (bin && relabeled)
                KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<false, true, true, true>), cg, kCW, 0, C, Bn);
            else if (bin)
                KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<false, true, false, true>), cg, kCW, 0, C, Bn);
            else if (append && relabeled)
                KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<true, true, true>), cg, kCW, 0, C, Bn);
            else if (append)
                KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<true, true>), cg, kCW, 0, C, Bn);
            else if (relabeled)
                KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<false, true, true>), cg, kCW, 0, C, Bn);
            else
                KARMA_LAUNCH(ctx, "graph_classify", (classify2_kernel<false, true>), cg, kCW, 0, C, Bn);
            return KARMA_OK;
        };
        if (probe) {
            // a probe of the reads decides: when many span more than 4 contig
            // ids, this pass is skipped and a relabelled rerun follows
            KARMA_LAUNCH(ctx, "relabel_probe", relabel_probe_kernel, 1, kRelabelProbes, 0, rec, A, (uint32_t)N,
                         counters + 3, reinterpret_cast<uint64_t*>(cb), (int64_t)(ctrl_words + 2 * n_pblk + B));
            C.skip = counters + 3;
        } else if (fresh_ext) {
            C.skip = counters + 3;
            C.vote = counters + 4;
        }
        KARMA_TRY(classify(0, n_chunks));
    }
    // where side-stream work (the k-mer profile) may start: 5 = after the final
    // kernel, beside the control-block readback (default; 0.283 against 0.291
    // ms for the 8-rank strong preview, equal on one GPU, profiles/r03/measurements.md (ab_mark5)),
    // 0 = after the whole pipeline, 1 = after classify, 2 = after the code
    // partition, 3 = at once (beside classify), 4 = after the code reduce.
    // Measured: 1 slows the code partition 0.19 -> 0.5 ms (1.46 vs 1.37 ms/step);
    // 2 stretches the profile to 0.60 ms beside the reduce (1.43 vs 1.35);
    // 3 stretches classify 0.54 -> 0.74 ms (1.35 vs 1.25): HBM is already full
    auto mark = [&](int at) -> int {
        if (mark_at(ctx) != at || attempt != 0) return KARMA_OK;
        if (!ctx->mark_ev) KARMA_HIP(hipEventCreateWithFlags(&ctx->mark_ev, hipEventDisableTiming));
        KARMA_HIP(hipEventRecord(ctx->mark_ev, ctx->stream));
        ctx->mark_set = true;
        return KARMA_OK;
    };
    KARMA_TRY(mark(1));
    if (A == 0) {
        KARMA_HIP(hipMemsetAsync(n_codes.ptr, 0, n_chunks * 4, ctx->stream));
        KARMA_HIP(hipMemsetAsync(n_gen.ptr, 0, n_chunks * 4, ctx->stream));
        if (bin) KARMA_HIP(hipMemsetAsync(bhdr.ptr, 0, n_chunks * 16 * kBinHdr, ctx->stream));
    }
    const RunDir cdir{cf_base.ptr, cf_off.ptr, counters + 1, blk_items};
    pdir = RunDir{pf_base.ptr, pf_off.ptr, counters + 2, blk_items + n_pblk};
    // Two independent branches after classify, joined by the final kernel:
    // general reads -> pair lists -> pair partition -> pair reduce, and the
    // code partition -> code reduce.  The first (three short kernels) runs on
    // the context's fork stream beside the second.
    hipStream_t const main_stream = ctx->stream;
    // (not while every launch is timed: the per-kernel pass wants each kernel
    // alone on the chip)
    const bool fork = fork_on() && !ctx->no_fork && !(ctx->timing && ctx->timing_only.empty());
    hipStream_t fork_s = nullptr;  // set by ctx_fork: ctx->fork_use or ctx->fork_stream
    if (fork) {
        KARMA_TRY(ctx_fork(ctx));
        fork_s = ctx->fork_use ? ctx->fork_use : ctx->fork_stream;
        KARMA_HIP(hipEventRecord(ctx->fork_a, main_stream));
        KARMA_HIP(hipStreamWaitEvent(fork_s, ctx->fork_a, 0));
        ctx->stream = fork_s;
    }
    int rc_pair = [&]() -> int {
        KARMA_LAUNCH(ctx, "graph_general", general_kernel, general_grid(ctx, n_chunks), kGW, 0, rec, A, (uint32_t)N,
                     codes.ptr, n_gen.ptr, n_chunks, plist.ptr, pcap, n_pl.ptr, blk_items + n_pblk, lpb, flags,
                     relabeled ? (const uint32_t*)remap_map.ptr : nullptr, (const unsigned*)(counters + 3), chunk);
        if (wide_p)
            KARMA_LAUNCH(ctx, "graph_pair_partition", partition_kernel<PairStreamWide>, n_pblk, kPT, 0, plist.ptr,
                         pcap, n_pl.ptr, n_chunks, lpb, g, pent.ptr, pdir);
        else
            KARMA_LAUNCH(ctx, "graph_pair_partition", partition_kernel<PairStream>, n_pblk, kPT, 0, plist.ptr, pcap,
                         n_pl.ptr, n_chunks, lpb, g, pent.ptr, pdir);
        KARMA_LAUNCH(ctx, "graph_pair_reduce", pair_reduce_kernel, nsl, kRT, 0, pent.ptr, pdir, n_pg, g.bw, g.bbits,
                     g.dbits, B, part_b.ptr, part_k.ptr, part_c.ptr, part_n.ptr, ovf);
        if (fork) KARMA_HIP(hipEventRecord(ctx->fork_b, fork_s));
        return KARMA_OK;
    }();
    ctx->stream = main_stream;
    KARMA_TRY(rc_pair);
    if (bin) {
        KARMA_LAUNCH(ctx, "graph_code_reduce", code_seg_reduce_kernel, (int64_t)g.Bc * n_cg, kCRT, 0, bsegs.ptr,
                     reinterpret_cast<const uint4*>(bhdr.ptr), bdir.ptr, n_chunks, seg_cap, dir_cap, g.bwc, n_cg,
                     part_ch.ptr, back_list_cap(), slotted ? 1 : 0);
        // position 2 ("after the code partition": the profile beside the
        // LDS-bound reduce) is after the reduce here: its 132 KB blocks
        // cannot share a CU with the profile's, so a profile started after
        // classify ran first and the reduce after it (config 3 1.13 against
        // 1.05 ms per step)
        KARMA_TRY(mark(2));
    } else if (g.Bc > 0) {
        uint16_t* const trash = cent.ptr + (ccap + 7) / 8 * 8;
        if (append && wide_c)
            KARMA_LAUNCH(ctx, "graph_code_partition", code_append_kernel<kMaxBc>, n_pblk, kPT, 0, codes.ptr, chunk,
                         n_codes.ptr, n_chunks, lpb, g, blk_hist.ptr, cent.ptr, trash, cdir, flags + 3);
        else if (append)
            KARMA_LAUNCH(ctx, "graph_code_partition", code_append_kernel<kNarrowBc>, n_pblk, kPT, 0, codes.ptr,
                         chunk, n_codes.ptr, n_chunks, lpb, g, blk_hist.ptr, cent.ptr, trash, cdir, flags + 3);
        else if (wide_c)
            KARMA_LAUNCH(ctx, "graph_code_partition", partition_kernel<CodeStreamWide>, n_pblk, kPT, 0, codes.ptr,
                         chunk, n_codes.ptr, n_chunks, lpb, g, cent.ptr, cdir);
        else
            KARMA_LAUNCH(ctx, "graph_code_partition", partition_kernel<CodeStream>, n_pblk, kPT, 0, codes.ptr, chunk,
                         n_codes.ptr, n_chunks, lpb, g, cent.ptr, cdir);
        KARMA_TRY(mark(2));
        KARMA_LAUNCH(ctx, "graph_code_reduce", code_reduce_kernel, (int64_t)g.Bc * n_cg, kCRT, 0, cent.ptr, cdir,
                     g.Bc, g.bwc, n_cg, part_ch.ptr);
    }
    KARMA_TRY(mark(4));  // after the code reduce: beside the final kernel
    if (fork) KARMA_HIP(hipStreamWaitEvent(main_stream, ctx->fork_b, 0));
    SplitArgs sa{};
    sa.n = (int)split_b.size();
    for (int r = 0; r < sa.n; ++r) sa.b[r] = split_b[r];
    sa.out = split_loc;
    if (n_pg == 1)
        KARMA_LAUNCH(ctx, "graph_bucket_final", final_kernel<kHashR>, B, kFT, 0, n_pg, n_cg, g.bw, g.bbits, g.dbits,
                     g.bwc, part_b.ptr, part_ch.ptr, part_k.ptr, part_c.ptr, part_n.ptr, slot_k.ptr, slot_c.ptr, n_per,
                     ovf, sa, lb, dst);
    else
        KARMA_LAUNCH(ctx, "graph_bucket_final", final_kernel<kHashF>, B, kFT, 0, n_pg, n_cg, g.bw, g.bbits, g.dbits,
                     g.bwc, part_b.ptr, part_ch.ptr, part_k.ptr, part_c.ptr, part_n.ptr, slot_k.ptr, slot_c.ptr, n_per,
                     ovf, sa, lb, dst);
    KARMA_TRY(mark(5));  // after the final kernel, before the control-block readback
    if (!deferred)
        KARMA_HIP(hipMemcpyAsync(const_cast<int64_t*>(hctrl), cb, ctrl_words * 8, hipMemcpyDeviceToHost,
                                 ctx->stream));
    return KARMA_OK;
}

int SetsJob::relabel() {
    const uint32_t n = (uint32_t)N;
    DevArray<uint32_t> rep, root;
    DevArray<unsigned> fill;
    DevArray<int64_t> size, base;
    KARMA_TRY(remap_map.alloc(ctx, N));
    KARMA_TRY(remap_inv.alloc(ctx, N));
    KARMA_TRY(rep.alloc(ctx, N));
    KARMA_TRY(root.alloc(ctx, N));
    KARMA_TRY(fill.alloc(ctx, N));
    KARMA_TRY(size.alloc(ctx, N + 1));
    KARMA_TRY(base.alloc(ctx, N + 1));
    KARMA_LAUNCH(ctx, "relabel_iota", iota_u32_kernel, grid_n(N), 256, 0, rep.ptr, N);
    // hooks from a sample of the reads (the records' first 1/32, >= 4M
    // records): a gene's contigs join through a few of its reads, and a contig
    // left out only keeps its (few) reads on the general path
    const int64_t As = std::min<int64_t>(A, std::max<int64_t>(A / 32, int64_t(1) << 22));
    if (As) KARMA_LAUNCH(ctx, "relabel_hook", relabel_hook_kernel, grid_n(As), 256, 0, rec, As, n, rep.ptr);
    KARMA_HIP(hipMemsetAsync(size.ptr, 0, (N + 1) * 8, ctx->stream));
    KARMA_HIP(hipMemsetAsync(fill.ptr, 0, N * 4, ctx->stream));
    KARMA_LAUNCH(ctx, "relabel_root", relabel_root_kernel, grid_n(N + 1), 256, 0, rep.ptr, n, root.ptr, size.ptr);
    KARMA_TRY(scan_excl_i64(ctx, size.ptr, base.ptr, N + 1));
    KARMA_LAUNCH(ctx, "relabel_assign", relabel_assign_kernel, grid_n(N), 256, 0, root.ptr, base.ptr, n, fill.ptr,
                 remap_map.ptr, remap_inv.ptr);
    return KARMA_OK;
}

int SetsJob::finish(karma_pairs* out) {
    unsigned hc[4] = {0, 0, 0, 0};
    std::vector<uint8_t> hovf(B);
    int64_t U = 0;
    for (;;) {
        // the one synchronisation of the common path
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
        const int* hf = reinterpret_cast<const int*>(hctrl);
        std::memcpy(hc, hctrl + 2, sizeof hc);
        std::memcpy(hovf.data(), hctrl + 6 + 2 * (B + 1), B);
        U = hctrl[6 + (B + 1) + B];
        KARMA_CHECK(!hf[0], KARMA_ERR_UNSORTED, "records are not grouped by read (read ids decrease)");
        KARMA_CHECK(!hf[1], KARMA_ERR_ARG, "a record's contig index is >= n_contigs (%lld)", (long long)N);
        KARMA_CHECK(!hf[3], KARMA_ERR_STATE, "code partition: block counts disagree with the classify histogram");
        if (!relabeled && hc[3]) {  // most reads were general: rerun on relabelled contigs
            KARMA_TRY(relabel());
            relabeled = true;
            KARMA_TRY(launch());
            continue;
        }
        if (!hf[2]) break;
        KARMA_CHECK(attempt == 0, KARMA_ERR_STATE, "pair list capacity exceeded twice");
        attempt = 1;
        pcap = chunk * 9 / 2;  // every read with <= 8 records fits
        KARMA_TRY(launch());
    }
    const unsigned n_big = hc[0];
    if (std::getenv("KARMA_DEBUG_GEN")) {  // diagnostic: reads on the general path, big reads
        std::vector<uint32_t> hg(n_chunks);
        KARMA_HIP(hipMemcpy(hg.data(), n_gen.ptr, n_chunks * 4, hipMemcpyDeviceToHost));
        uint64_t tot = 0;
        for (uint32_t x : hg) tot += x;
        std::fprintf(stderr, "[karma] general reads %llu, big reads %u, pair flushes %u\n", (unsigned long long)tot,
                     n_big, hc[2]);
    }
    DevArray<const uint64_t*> pk;  // per-bucket list overrides (overflowed buckets only)
    DevArray<const int64_t*> pc;
    DevArray<int64_t> src_off;     // where the final kernel put each other bucket's list
    std::vector<std::unique_ptr<DevArray<uint64_t>>> keep_k;
    std::vector<std::unique_ptr<DevArray<int64_t>>> keep_c;
    const int64_t widen_threads = std::max<int64_t>(hc[2], (int64_t(8) << g.bw) + 24);
    bool any_ovf = false;
    for (int b = 0; b < B; ++b) {
        if (!hovf[b]) continue;
        if (!any_ovf) {
            KARMA_TRY(pk.alloc(ctx, B));
            KARMA_TRY(pc.alloc(ctx, B));
            KARMA_TRY(src_off.alloc(ctx, B));
            KARMA_HIP(hipMemcpyAsync(src_off.ptr, dst, B * 8, hipMemcpyDeviceToDevice, ctx->stream));
            KARMA_HIP(hipMemsetAsync(pk.ptr, 0, B * sizeof(void*), ctx->stream));
            KARMA_HIP(hipMemsetAsync(pc.ptr, 0, B * sizeof(void*), ctx->stream));
        }
        any_ovf = true;
        // generic path for a bucket whose distinct pairs exceed the LDS tables
        DevArray<unsigned long long> np;
        KARMA_TRY(np.alloc(ctx, 1));
        KARMA_HIP(hipMemsetAsync(np.ptr, 0, 8, ctx->stream));
        KARMA_LAUNCH(ctx, "bucket_widen", bucket_widen_kernel, grid_n(widen_threads, 64), 64, 0, pent.ptr, pdir, B,
                     b, g.bw, g.bbits, part_ch.ptr, n_cg, g.bwc, (uint64_t*)nullptr, (int64_t*)nullptr, np.ptr, 1);
        unsigned long long hp = 0;
        KARMA_HIP(hipMemcpyAsync(&hp, np.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
        DevArray<uint64_t> wide;
        DevArray<int64_t> wc;
        KARMA_TRY(wide.alloc(ctx, hp));
        KARMA_TRY(wc.alloc(ctx, hp));
        KARMA_HIP(hipMemsetAsync(np.ptr, 0, 8, ctx->stream));
        KARMA_LAUNCH(ctx, "bucket_widen", bucket_widen_kernel, grid_n(widen_threads, 64), 64, 0, pent.ptr, pdir, B,
                     b, g.bw, g.bbits, part_ch.ptr, n_cg, g.bwc, wide.ptr, wc.ptr, np.ptr, 0);
        keep_k.emplace_back(new DevArray<uint64_t>());
        keep_c.emplace_back(new DevArray<int64_t>());
        int64_t nu = 0;
        KARMA_TRY(sort_reduce_pairs(ctx, wide.ptr, wc.ptr, nullptr, (int64_t)hp, 64, *keep_k.back(), *keep_c.back(),
                                    nullptr, &nu));
        const uint64_t* kp = keep_k.back()->ptr;
        const int64_t* cp = keep_c.back()->ptr;
        KARMA_HIP(hipMemcpyAsync(pk.ptr + b, &kp, sizeof kp, hipMemcpyHostToDevice, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(pc.ptr + b, &cp, sizeof cp, hipMemcpyHostToDevice, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(n_per + b, &nu, 8, hipMemcpyHostToDevice, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
    }
    if (any_ovf) {
        KARMA_TRY(scan_excl_i64(ctx, n_per, dst, B + 1));
        KARMA_HIP(hipMemcpyAsync(&U, dst + B, 8, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
    }
    DevArray<uint64_t> mk;
    DevArray<int64_t> mc;
    if (any_ovf) {
        KARMA_TRY(mk.alloc(ctx, U));
        KARMA_TRY(mc.alloc(ctx, U));
        KARMA_LAUNCH(ctx, "bucket_assemble", assemble2_kernel, B, 256, 0, slot_k.ptr, slot_c.ptr, src_off.ptr,
                     pk.ptr, pc.ptr, n_per, dst, mk.ptr, mc.ptr);
    } else {
        // the final kernel wrote the buckets' lists back to back: the list as is
        // (its arrays hold B x kSlotCap entries, the first U of them used)
        mk.swap(slot_k);
        mc.swap(slot_c);
    }
    if (!relabeled) {
        KARMA_TRY(finish_pairs(ctx, rec, A, N, big_list.ptr, n_big, mk, mc, U, out));
        if (!split_b.empty() && !any_ovf && n_big == 0) {
            // the owners' slice starts, from the final kernel's in-bucket counts
            const int64_t* h_dst = hctrl + 6 + (B + 1);
            const int64_t* h_loc = h_dst + (B + 1) + ceil_div(B, 8);
            out->split_bounds = split_b;
            out->split_starts.resize(split_b.size());
            for (size_t r = 0; r < split_b.size(); ++r) {
                const int64_t b = split_b[r] >> g.bw;
                out->split_starts[r] = split_b[r] <= 0 ? 0 : (b < B ? h_dst[b] + h_loc[r] : U);
            }
        }
        return KARMA_OK;
    }
    KARMA_TRY(finish_pairs(ctx, rec, A, N, big_list.ptr, n_big, mk, mc, U, out, remap_map.ptr));
    // back to the original ids, sorted again (keys stay unique: the map is a bijection)
    if (out->n) KARMA_LAUNCH(ctx, "relabel_back", relabel_back_kernel, grid_n(out->n), 256, 0, out->keys.ptr, out->n,
                             remap_inv.ptr);
    DevArray<uint64_t> k2;
    DevArray<int64_t> c2;
    int64_t n2 = 0;
    KARMA_TRY(sort_reduce_pairs(ctx, out->keys.ptr, out->counts.ptr, nullptr, out->n, 64, k2, c2, nullptr, &n2));
    out->keys.swap(k2);
    out->counts.swap(c2);
    out->n = n2;
    return KARMA_OK;
}

int64_t sets_max_contigs() { return kMaxCompactN; }

int sets_begin(karma_ctx* ctx, RecIn rec, int64_t A, int64_t N, SetsJob** job) {
    KARMA_CHECK(N <= kMaxCompactN, KARMA_ERR_ARG, "sets_begin: n_contigs above the compact path");
    KARMA_CHECK(!ctx->job_open, KARMA_ERR_STATE, "a split graph call is already open on this context");
    std::unique_ptr<SetsJob> j(new SetsJob());
    j->ctx = ctx;
    j->rec = rec;
    j->A = A;
    j->N = N;
    if (!ctx->split_bounds.empty() && (int)ctx->split_bounds.size() <= kMaxSplit) j->split_b = ctx->split_bounds;
    ctx->split_bounds.clear();  // one job
    KARMA_TRY(j->setup());
    const int rc = j->launch();
    if (rc) {
        ctx->mark_set = false;
        return rc;
    }
    ctx->job_open = true;
    *job = j.release();
    return KARMA_OK;
}

int sets_end(SetsJob* job, karma_pairs* out) {
    std::unique_ptr<SetsJob> j(job);
    j->ctx->job_open = false;
    j->ctx->mark_set = false;
    return j->finish(out);
}

void sets_free(SetsJob* job) {
    if (!job) return;
    job->ctx->job_open = false;
    job->ctx->mark_set = false;
    hipStreamSynchronize(job->ctx->stream);  // its kernels may still use the scratch
    delete job;
}

int sets_begin_deferred(karma_ctx* ctx, RecIn rec, int64_t A, int64_t N, SetsJob** job, SetsDeferred* v) {
    KARMA_CHECK(N <= kMaxCompactN, KARMA_ERR_ARG, "sets_begin: n_contigs above the compact path");
    KARMA_CHECK(!ctx->job_open, KARMA_ERR_STATE, "a split graph call is already open on this context");
    std::unique_ptr<SetsJob> j(new SetsJob());
    j->ctx = ctx;
    j->rec = rec;
    j->A = A;
    j->N = N;
    j->deferred = true;
    if (!ctx->split_bounds.empty() && (int)ctx->split_bounds.size() <= kMaxSplit) j->split_b = ctx->split_bounds;
    ctx->split_bounds.clear();  // one job
    KARMA_TRY(j->setup());
    const int rc = j->launch();
    if (rc) {
        ctx->mark_set = false;
        return rc;
    }
    v->keys = j->slot_k.ptr;
    v->counts = j->slot_c.ptr;
    v->cap = (int64_t)j->B * kSlotCap;
    v->dst = j->dst;
    v->split_loc = j->split_loc;
    v->split_b = j->split_b;
    v->B = j->B;
    v->bw = j->g.bw;
    v->flags = j->flags;
    v->counters = j->counters;
    v->ovf = j->ovf;
    v->ctrl = j->ext ? j->cb : nullptr;
    v->ctrl_need = j->ctrl_words + 2 * j->n_pblk + j->B;
    ctx->job_open = true;
    *job = j.release();
    return KARMA_OK;
}

void sets_release(SetsJob* job) {
    if (!job) return;
    job->ctx->job_open = false;
    job->ctx->mark_set = false;
    delete job;  // its buffers go back to the main stream's cache: later work there is ordered after its kernels
}

int records_to_pairs_sets(karma_ctx* ctx, RecIn rec, int64_t A, int64_t N, karma_pairs* out) {
    if (N > kMaxCompactN) return records_to_pairs_wide(ctx, rec, A, N, out);
    SetsJob* job = nullptr;
    KARMA_TRY(sets_begin(ctx, rec, A, N, &job));
    return sets_end(job, out);
}

}  // namespace karma
