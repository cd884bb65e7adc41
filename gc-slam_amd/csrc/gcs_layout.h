// Device data layout shared by kernels and host code (DESIGN.md "Data layout in HBM").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gcs {

// ScanBinStats (archive/legacy_operators/binning.py:40-48) as 26 field-major f64 arrays of
// length B: field f of bin b lives at scan[f * B + b] (coalesced per-bin streaming).
enum ScanField : int {
  SF_N = 0,       // N (mass)
  SF_SD = 1,      // s_dir[3]
  SF_S = 4,       // S_dir_scatter[3][3]
  SF_PB = 13,     // p_bar[3]
  SF_SIG = 16,    // Sigma_p[3][3]
  SF_KAPPA = 25,  // kappa_scan
  SF_COUNT = 26
};

// MapBinStats sufficient statistics (archive/bin_atlas.py:83-101), field-major.
enum MapField : int {
  MF_SD = 0,     // S_dir[3]
  MF_S = 3,      // S_dir_scatter[3][3]
  MF_ND = 12,    // N_dir
  MF_NP = 13,    // N_pos
  MF_SP = 14,    // sum_p[3]
  MF_SPP = 17,   // sum_ppT[3][3]
  MF_COUNT = 26
};

// MapDerivedStats (archive/bin_atlas.py:104-114), field-major.
enum MapDerived : int {
  MD_MU = 0,     // mu_dir[3]
  MD_KAPPA = 3,  // kappa
  MD_C = 4,      // centroid[3]
  MD_SIG = 7,    // Sigma_c[3][3]
  MD_COUNT = 16
};

// Per-point record written by the point kernel, gathered by the bin kernels (64 B, exactly what the
// bin kernel stages in LDS: four 16-B loads per record).
struct PointRec {
  double x, y, z;     // deskewed point (scan-start base frame)
  double dx, dy, dz;  // ray direction from the LiDAR origin (pipeline.py:589-593)
  double m;           // max candidate similarity (softmax shift)
  double wz;          // w / Z: weight after budget mass rescale and deskew time window (w), times
                      // 1 / Z, Z = sum_k exp((s_k - m) / tau); w r_k = wz exp((s_k - m) / tau)
};
static_assert(sizeof(PointRec) == 64, "point record");

// Scale mode's point record (round 6): the deskewed point and w / Z only.  The bin kernel's staging
// recomputes the other two fields bit for bit: d = ray_dir(p) (the point kernel's own expression), and
// the softmax shift m, which is the dot of d with the point's nearest bin -- the record's source bucket
// -- because that bin maximises the exact dot over the whole atlas and is one of its own K candidates.
// Half the bytes the point kernel writes and every bin tile fed by the bucket re-reads.
struct PointRec32 {
  double x, y, z;  // deskewed point (scan-start base frame)
  double wz;       // w / Z as in PointRec
};
static_assert(sizeof(PointRec32) == 32, "scale-mode point record");

// Scalar results slots (device buffer of doubles, copied to host once per scan).
enum Scalar : int {
  SC_MASS_IN = 0,       // sum w (raw)
  SC_MASS_SEL = 1,      // sum w over stride-selected rows
  SC_MASS_SCALE = 2,
  SC_DESKEW_WIN = 3,    // sum budget weights (deskew input)
  SC_BUDGET_W2 = 4,     // sum (w_budget/(mass_in+eps))^2
  SC_DESKEW_WOUT = 5,   // sum deskewed weights
  SC_ENTROPY = 6,       // sum_n H_n
  SC_MAXRESP = 7,       // max r
  SC_BIN_NSUM = 8,      // sum_b N_b
  SC_BIN_N2SUM = 9,     // sum_b N_b^2
  SC_BIN_SUPP = 10,     // sum_b N_b/(N_b+eps)
  SC_BIN_PSD = 11,      // sum_b psd projection delta
  SC_BIN_EPSR = 12,     // max_b eps ratio
  SC_MF_H = 16,         // H[9]
  SC_MF_NEFF = 25,
  SC_MF_MAPSCAT = 26,   // sum_b map S_dir_scatter [9]
  SC_MF_MAPND = 35,     // sum_b map N_dir
  SC_MF_SCANN = 36,     // sum_b scan N
  SC_MF_MAPN = 37,      // sum_b map N_dir (alias, kept for cert)
  SC_MF_R = 40,         // R_mf[9] (device SVD result)
  SC_MF_S = 49,         // singular values [3]
  SC_MF_V = 52,         // V[9] (columns = right singular vectors)
  SC_PT_L = 64,         // L_full[9]
  SC_PT_H = 73,         // h_full[3]
  SC_PT_NEFF = 76,
  SC_COUNT = 96
};

// The scan's host mirror (pinned, coherent, mapped): the PT fold copies the scalar block and the
// four device error words into it, then the scan's sequence number and a checksum of all of it.
// The host accepts the mirror only when the sequence word is the scan's and the checksum of what it
// reads matches (gcs_capi.cpp wait_mirror), so a read that overtakes any of the device's stores is
// re-read, never consumed -- whatever order the stores reach host memory in.
enum Mirror : int {
  MIR_ERR = SC_COUNT,      // 2 words: error words [0..1] | [2..3] (uint32 pairs)
  MIR_SEQ = SC_COUNT + 2,  // uint64 sequence number of the scan that wrote the mirror
  MIR_SUM = SC_COUNT + 3,  // uint64 checksum of words [0, MIR_SEQ] (mirror_word_hash summed) + seq
  MIR_WORDS = SC_COUNT + 4
};
// splitmix64's finalizer over (word + position x golden ratio): a torn mirror (any subset of stale
// words) sums to the fresh checksum with probability ~2^-64
__host__ __device__ inline uint64_t mirror_word_hash(uint64_t w, uint32_t i) {
  uint64_t z = w + 0x9e3779b97f4a7c15ULL * (uint64_t)(i + 1);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

}  // namespace gcs
