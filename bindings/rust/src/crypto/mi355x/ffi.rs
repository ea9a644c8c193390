//! Raw declarations of `include/sda_engine.h` (ABI version 1), one to one: same names, same argument
//! order, same integer widths.  `tests/test_rust_ffi.py` parses this `extern "C"` block and the C header
//! and fails on any difference.  UNCOMPILED here (the image has no cargo / rustc).
#![allow(non_camel_case_types, dead_code)]

use libc::{c_char, c_int, c_void};

pub const SDA_ENGINE_ABI_VERSION: c_int = 1;

/// `sda_status` (include/sda_engine.h); 1..=6 are the reference's error strings.
pub type SdaStatus = c_int;
pub const SDA_OK: SdaStatus = 0;
pub const SDA_ERR_BATCH_INPUT_WRONG_LENGTH: SdaStatus = 1;      // additive.rs:33
pub const SDA_ERR_PACKED_SHARING_FAILED: SdaStatus = 2;         // packed_shamir.rs:41
pub const SDA_ERR_WRONG_DIMENSION: SdaStatus = 3;               // combiner.rs:21
pub const SDA_ERR_MISMATCHING_DIMENSION: SdaStatus = 4;         // additive.rs:64
pub const SDA_ERR_INPUTS_MUST_HAVE_SAME_LENGTH: SdaStatus = 5;  // packed_shamir.rs:74
pub const SDA_ERR_NOT_ENOUGH_SHARES: SdaStatus = 6;             // packed_shamir.rs:75
pub const SDA_ERR_PRECONDITION: SdaStatus = 64;                 // where the reference panics
pub const SDA_ERR_INVALID_ARGUMENT: SdaStatus = 65;
pub const SDA_ERR_UNSUPPORTED: SdaStatus = 66;
pub const SDA_ERR_DEVICE: SdaStatus = 67;
pub const SDA_ERR_OUT_OF_MEMORY: SdaStatus = 68;

pub const SDA_SHARING_ADDITIVE: i32 = 0;
pub const SDA_SHARING_PACKED_SHAMIR: i32 = 1;
pub const SDA_MASKING_NONE: i32 = 0;
pub const SDA_MASKING_FULL: i32 = 1;
pub const SDA_MASKING_CHACHA: i32 = 2;
pub const SDA_REVEAL_EXACT: i32 = 0;
pub const SDA_REVEAL_CANONICAL: i32 = 1;

/// `sda_sharing_scheme`: protocol/src/crypto.rs:79-114 LinearSecretSharingScheme.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct SdaSharingScheme {
    pub kind: i32,
    pub share_count: u64,
    pub modulus: i64,
    pub secret_count: u64,
    pub privacy_threshold: u64,
    pub omega_secrets: i64,
    pub omega_shares: i64,
}

/// `sda_masking_scheme`: protocol/src/crypto.rs:43-64 LinearMaskingScheme.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct SdaMaskingScheme {
    pub kind: i32,
    pub modulus: i64,
    pub dimension: u64,
    pub seed_bitsize: u64,
}

/// Opaque `sda_engine`.
#[repr(C)]
pub struct SdaEngine {
    _private: [u8; 0],
}

#[link(name = "sda_engine")]
extern "C" {
    // ---- lifecycle / diagnostics ----
    pub fn sda_abi_version() -> c_int;
    pub fn sda_engine_create(device_ordinal: c_int, out: *mut *mut SdaEngine) -> SdaStatus;
    pub fn sda_engine_destroy(h: *mut SdaEngine);
    pub fn sda_engine_synchronize(h: *mut SdaEngine) -> SdaStatus;
    pub fn sda_engine_create_multi(ordinals: *const c_int, n_devices: c_int, out: *mut *mut SdaEngine) -> SdaStatus;
    pub fn sda_engine_device_count(h: *const SdaEngine) -> c_int;
    pub fn sda_last_error_message() -> *const c_char;
    pub fn sda_status_string(status: c_int) -> *const c_char;

    // ---- derived scheme sizes: protocol/src/crypto.rs:117-155 ----
    pub fn sda_scheme_input_size(s: *const SdaSharingScheme) -> u64;
    pub fn sda_scheme_output_size(s: *const SdaSharingScheme) -> u64;
    pub fn sda_scheme_privacy_threshold(s: *const SdaSharingScheme) -> u64;
    pub fn sda_scheme_reconstruction_threshold(s: *const SdaSharingScheme) -> u64;
    pub fn sda_share_length(s: *const SdaSharingScheme, dimension: u64) -> u64;

    // ---- trait mirrors (host buffers, synchronous) ----
    pub fn sda_share_generate(h: *mut SdaEngine, s: *const SdaSharingScheme, secrets: *const i64, dimension: u64,
                              draws: *const i64, n_draws: u64, out: *mut i64, out_cap: u64) -> SdaStatus;
    pub fn sda_share_combine(h: *mut SdaEngine, s: *const SdaSharingScheme, rows: *const *const i64,
                             lens: *const u64, n_rows: u64, out: *mut i64, out_cap: u64, out_len: *mut u64)
                             -> SdaStatus;
    pub fn sda_secret_reconstruct(h: *mut SdaEngine, s: *const SdaSharingScheme, dimension: u64,
                                  indices: *const u64, rows: *const *const i64, lens: *const u64, n_rows: u64,
                                  out: *mut i64, out_cap: u64, out_len: *mut u64) -> SdaStatus;
    pub fn sda_secret_mask(h: *mut SdaEngine, s: *const SdaMaskingScheme, secrets: *const i64, dimension: u64,
                           seed: *const u32, seed_words: u64, full_masks: *const i64, mask_out: *mut i64,
                           mask_cap: u64, mask_len: *mut u64, masked_out: *mut i64) -> SdaStatus;
    pub fn sda_mask_combine(h: *mut SdaEngine, s: *const SdaMaskingScheme, rows: *const *const i64,
                            lens: *const u64, n_rows: u64, out: *mut i64, out_cap: u64, out_len: *mut u64)
                            -> SdaStatus;
    pub fn sda_secret_unmask(h: *mut SdaEngine, s: *const SdaMaskingScheme, mask: *const i64, mask_len: u64,
                             masked: *const i64, masked_len: u64, out: *mut i64, out_cap: u64, out_len: *mut u64)
                             -> SdaStatus;
    pub fn sda_recipient_positive(h: *mut SdaEngine, modulus: i64, values: *const i64, n: u64, out: *mut i64)
                                  -> SdaStatus;

    // ---- device-resident entry points ----
    pub fn sda_combine_dev(h: *mut SdaEngine, modulus: i64, shares: *const i64, n: u64, dim: u64, row_stride: u64,
                           out: *mut i64, stream: *mut c_void) -> SdaStatus;
    pub fn sda_combine_accumulate_dev(h: *mut SdaEngine, modulus: i64, shares: *const i64, n: u64, dim: u64,
                                      row_stride: u64, inout: *mut i64, stream: *mut c_void) -> SdaStatus;
    pub fn sda_combine_finalize_dev(h: *mut SdaEngine, modulus: i64, sums: *const i64, dim: u64, out: *mut i64,
                                    stream: *mut c_void) -> SdaStatus;
    pub fn sda_combine_split_dev(h: *mut SdaEngine, modulus: i64, shares: *const i64, n: u64, dim: u64,
                                 row_stride: u64, inout: *mut i64, flags: *mut i64, stream: *mut c_void)
                                 -> SdaStatus;
    pub fn sda_combine_split_prefix_dev(h: *mut SdaEngine, modulus: i64, gathered: *const i64, world: u64,
                                        rank: u64, dim: u64, c_in: *mut i64, total: *mut i64, code: *mut i32,
                                        stream: *mut c_void) -> SdaStatus;
    pub fn sda_combine_split_replay_dev(h: *mut SdaEngine, modulus: i64, shares: *const i64, n: u64, dim: u64,
                                        row_stride: u64, rank: u64, state: *mut i64, code: *mut i32,
                                        stream: *mut c_void) -> SdaStatus;
    pub fn sda_combine_split_resolve_dev(h: *mut SdaEngine, modulus: i64, total: *const i64, code: *const i32,
                                         dim: u64, out: *mut i64, stream: *mut c_void) -> SdaStatus;
    pub fn sda_packed_generate_dev(h: *mut SdaEngine, s: *const SdaSharingScheme, secrets: *const i64,
                                   dimension: u64, n_vectors: u64, draws: *const i64, out: *mut i64,
                                   stream: *mut c_void) -> SdaStatus;
    pub fn sda_packed_generate_mode_dev(h: *mut SdaEngine, s: *const SdaSharingScheme, secrets: *const i64,
                                        dimension: u64, n_vectors: u64, draws: *const i64, out: *mut i64,
                                        mode: i32, stream: *mut c_void) -> SdaStatus;
    pub fn sda_packed_reconstruct_dev(h: *mut SdaEngine, s: *const SdaSharingScheme, dimension: u64,
                                      indices: *const u64, n_idx: u64, n_vectors: u64, shares: *const i64,
                                      out: *mut i64, mode: i32, stream: *mut c_void) -> SdaStatus;
    pub fn sda_additive_generate_dev(h: *mut SdaEngine, modulus: i64, share_count: u64, secrets: *const i64,
                                     dimension: u64, draws: *const i64, out: *mut i64, stream: *mut c_void)
                                     -> SdaStatus;
    pub fn sda_chacha_mask_combine_dev(h: *mut SdaEngine, modulus: i64, dimension: u64, seeds: *const u32, w: u64,
                                       n_seeds: u64, out: *mut i64, stream: *mut c_void) -> SdaStatus;

    // ---- share payload codec (sodium.rs:36-41, :82-88) ----
    pub fn sda_varint_encode(h: *mut SdaEngine, vals: *const i64, n: u64, out: *mut u8, out_cap: u64,
                             out_len: *mut u64) -> SdaStatus;
    pub fn sda_varint_decode(h: *mut SdaEngine, bytes: *const u8, n_bytes: u64, out: *mut i64, out_cap: u64,
                             out_len: *mut u64) -> SdaStatus;
    pub fn sda_clerk_decode_combine(h: *mut SdaEngine, s: *const SdaSharingScheme, blobs: *const *const u8,
                                    blob_lens: *const u64, n_blobs: u64, out: *mut i64, out_cap: u64,
                                    out_len: *mut u64) -> SdaStatus;
    pub fn sda_varint_decode_dev(h: *mut SdaEngine, bytes: *const u8, blob_off: *const u64, n_blobs: u64,
                                 out: *mut i64, out_stride: u64, counts: *mut u64, stream: *mut c_void)
                                 -> SdaStatus;
    pub fn sda_clerk_decode_combine_dev(h: *mut SdaEngine, modulus: i64, bytes: *const u8, blob_off: *const u64,
                                        n_blobs: u64, out: *mut i64, out_cap: u64, out_len: *mut u64,
                                        stream: *mut c_void) -> SdaStatus;
    pub fn sda_varint_encode_dev(h: *mut SdaEngine, vals: *const i64, rows: u64, len: u64, stride: u64,
                                 dst: *mut u8, dst_cap: u64, row_bytes: *mut u64, stream: *mut c_void) -> SdaStatus;

    // ---- snapshot transposition (server/src/stores.rs:86-101) ----
    pub fn sda_snapshot_transpose_dev(h: *mut SdaEngine, src: *const u8, part_off: *const u64,
                                      n_participations: u64, n_clerks: u64, dst: *mut u8, dst_cap: u64,
                                      dst_len: *mut u64, clerk_base: *mut u64, clerk_off: *mut u64,
                                      stream: *mut c_void) -> SdaStatus;

    // ---- fused role pipelines ----
    pub fn sda_recipient_reveal_dev(h: *mut SdaEngine, ms: *const SdaMaskingScheme, mask_in: *const c_void,
                                    n_masks: u64, mask_width: u64, ss: *const SdaSharingScheme, dimension: u64,
                                    indices: *const u64, shares: *const i64, n_idx: u64, share_len: u64,
                                    output_modulus: i64, mode: i32, out: *mut i64, out_cap: u64,
                                    out_len: *mut u64, stream: *mut c_void) -> SdaStatus;
    pub fn sda_recipient_reveal(h: *mut SdaEngine, ms: *const SdaMaskingScheme, mask_rows: *const *const i64,
                                mask_lens: *const u64, n_masks: u64, ss: *const SdaSharingScheme, dimension: u64,
                                indices: *const u64, share_rows: *const *const i64, share_lens: *const u64,
                                n_idx: u64, output_modulus: i64, mode: i32, out: *mut i64, out_cap: u64,
                                out_len: *mut u64) -> SdaStatus;
    pub fn sda_participant_share_dev(h: *mut SdaEngine, ms: *const SdaMaskingScheme, seed: *const u32,
                                     seed_words: u64, full_masks: *const i64, ss: *const SdaSharingScheme,
                                     secrets: *const i64, dimension: u64, draws: *const i64, mode: i32,
                                     shares_out: *mut i64, payload: *mut u8, payload_cap: u64,
                                     payload_row_bytes: *mut u64, stream: *mut c_void) -> SdaStatus;

    // ---- synthetic benchmark input ----
    pub fn sda_synth_fill_dev(h: *mut SdaEngine, dst: *mut i64, rows: u64, cols: u64, seed: u64, lo: i64, hi: i64,
                              stream: *mut c_void) -> SdaStatus;

    // ---- HBM for resident buffers (fixed-size physical chunks) ----
    pub fn sda_hbm_alloc(device: c_int, bytes: u64, out: *mut *mut c_void) -> SdaStatus;
    pub fn sda_hbm_free(ptr: *mut c_void) -> SdaStatus;
    pub fn sda_hbm_trim(device: c_int, keep_bytes: u64) -> SdaStatus;
    pub fn sda_hbm_stats(device: c_int, live_bytes: *mut u64, pooled_bytes: *mut u64, retired_bytes: *mut u64)
        -> SdaStatus;
}
