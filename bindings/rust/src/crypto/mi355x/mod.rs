//! MI355X-backed implementations of the client's six crypto traits (client/src/crypto/sharing/mod.rs:14-33,
//! client/src/crypto/masking/mod.rs:13-31) over the C-ABI of `libsda_engine.so` (include/sda_engine.h).
//!
//! Drop this directory in as `client/src/crypto/mi355x/` and add `#[cfg(feature = "mi355x")] pub mod mi355x;`
//! to client/src/crypto/mod.rs; `factories.rs` holds the hooks the six factories call (README.md lists the
//! insertion points).  Randomness stays where the reference draws it: the shim takes its OsRng draws in the
//! reference's order and hands them to the engine, so a result depends only on (inputs, draws), exactly as
//! the reference's does.
//!
//! UNCOMPILED: this environment has no cargo / rustc.  tests/test_rust_ffi.py checks `ffi.rs` against the C
//! header; the same ABI calls run end to end from C (tests/abi_c/full_loop.c) and Python (sda_amd/engine.py).

pub mod factories;
pub mod ffi;

use self::ffi::*;
use super::*;
use rand::distributions::{IndependentSample, Range};
use rand::{OsRng, Rng};
use std::ffi::CStr;
use std::sync::{Arc, Mutex};

/// One engine handle (device ordinal, streams, scratch).  The engine orders a handle's calls itself; the
/// mutex serialises host threads, since the trait objects may be shared behind `&self`.
pub struct Device {
    h: Mutex<*mut SdaEngine>,
}

unsafe impl Send for Device {}
unsafe impl Sync for Device {}

impl Drop for Device {
    fn drop(&mut self) {
        let h = *self.h.lock().unwrap();
        unsafe { sda_engine_destroy(h) }
    }
}

impl Device {
    pub fn open(ordinal: i32) -> SdaClientResult<Arc<Device>> {
        if unsafe { sda_abi_version() } != SDA_ENGINE_ABI_VERSION {
            Err("libsda_engine ABI version mismatch")?
        }
        let mut h = std::ptr::null_mut();
        check(unsafe { sda_engine_create(ordinal, &mut h) })?;
        Ok(Arc::new(Device { h: Mutex::new(h) }))
    }

    /// One handle over several GPUs (sda_engine_create_multi): the trait calls split their work over them
    /// (a clerk's combine by columns, the recipient's ChaCha mask combine by seeds + one RCCL reduce) and
    /// still return when the result is in host memory.
    pub fn open_multi(ordinals: &[i32]) -> SdaClientResult<Arc<Device>> {
        if unsafe { sda_abi_version() } != SDA_ENGINE_ABI_VERSION {
            Err("libsda_engine ABI version mismatch")?
        }
        let mut h = std::ptr::null_mut();
        check(unsafe { sda_engine_create_multi(ordinals.as_ptr(), ordinals.len() as i32, &mut h) })?;
        Ok(Arc::new(Device { h: Mutex::new(h) }))
    }

    fn call<F: FnOnce(*mut SdaEngine) -> SdaStatus>(&self, f: F) -> SdaClientResult<()> {
        let h = self.h.lock().unwrap();
        check(f(*h))
    }
}

/// SDA_OK -> Ok; 1..=6 -> the reference's own error strings (`Err("Wrong dimension")` ...);
/// SDA_ERR_PRECONDITION -> panic, where the reference asserts (chacha.rs:26, none.rs:23 ...).
fn check(status: SdaStatus) -> SdaClientResult<()> {
    if status == SDA_OK {
        return Ok(());
    }
    let base = unsafe { CStr::from_ptr(sda_status_string(status)) }.to_string_lossy().into_owned();
    let detail = unsafe { CStr::from_ptr(sda_last_error_message()) }.to_string_lossy().into_owned();
    match status {
        1..=6 => Err(base)?,
        SDA_ERR_PRECONDITION => panic!("{}", detail),
        _ => Err(format!("{}: {}", base, detail))?,
    }
}

fn sharing_c(s: &LinearSecretSharingScheme) -> SdaSharingScheme {
    match *s {
        LinearSecretSharingScheme::Additive { share_count, modulus } => SdaSharingScheme {
            kind: SDA_SHARING_ADDITIVE,
            share_count: share_count as u64,
            modulus: modulus,
            secret_count: 0,
            privacy_threshold: 0,
            omega_secrets: 0,
            omega_shares: 0,
        },
        LinearSecretSharingScheme::PackedShamir {
            secret_count, share_count, privacy_threshold, prime_modulus, omega_secrets, omega_shares,
        } => SdaSharingScheme {
            kind: SDA_SHARING_PACKED_SHAMIR,
            share_count: share_count as u64,
            modulus: prime_modulus,
            secret_count: secret_count as u64,
            privacy_threshold: privacy_threshold as u64,
            omega_secrets: omega_secrets,
            omega_shares: omega_shares,
        },
    }
}

fn masking_c(s: &LinearMaskingScheme) -> SdaMaskingScheme {
    match *s {
        LinearMaskingScheme::None => SdaMaskingScheme { kind: SDA_MASKING_NONE, modulus: 0, dimension: 0, seed_bitsize: 0 },
        LinearMaskingScheme::Full { modulus } =>
            SdaMaskingScheme { kind: SDA_MASKING_FULL, modulus: modulus, dimension: 0, seed_bitsize: 0 },
        LinearMaskingScheme::ChaCha { modulus, dimension, seed_bitsize } => SdaMaskingScheme {
            kind: SDA_MASKING_CHACHA,
            modulus: modulus,
            dimension: dimension as u64,
            seed_bitsize: seed_bitsize as u64,
        },
    }
}

/// A `Vec<Vec<i64>>` as the (row pointers, row lengths) pair the ABI takes.
fn rows_of(v: &[Vec<i64>]) -> (Vec<*const i64>, Vec<u64>) {
    (v.iter().map(|r| r.as_ptr()).collect(), v.iter().map(|r| r.len() as u64).collect())
}

// ---------------------------------------------------------------- sharing

/// ShareGenerator + ShareCombiner for both LinearSecretSharingScheme variants.
pub struct GpuSharing {
    dev: Arc<Device>,
    scheme: LinearSecretSharingScheme,
    c: SdaSharingScheme,
    rng: OsRng,
}

impl GpuSharing {
    pub fn new(dev: Arc<Device>, scheme: &LinearSecretSharingScheme) -> GpuSharing {
        GpuSharing {
            dev: dev,
            scheme: scheme.clone(),
            c: sharing_c(scheme),
            rng: OsRng::new().expect("Unable to get randomness source"),
        }
    }

    /// The values the reference's RNG would draw for `dimension` secrets, in draw order:
    /// Additive: share_count - 1 `gen_range(0, m)` per secret (additive.rs:42-44);
    /// PackedShamir: privacy_threshold `Range::new(0, p - 1)` samples per batch (tss `share`).
    fn draws(&mut self, dimension: usize, batches: usize) -> Vec<i64> {
        match self.scheme {
            LinearSecretSharingScheme::Additive { share_count, modulus } => {
                let rng = &mut self.rng;
                (0..dimension * (share_count - 1)).map(|_| rng.gen_range(0_i64, modulus)).collect()
            }
            LinearSecretSharingScheme::PackedShamir { privacy_threshold, prime_modulus, .. } => {
                let range = Range::new(0, prime_modulus - 1);
                let rng = &mut self.rng;
                (0..batches * privacy_threshold).map(|_| range.ind_sample(rng)).collect()
            }
        }
    }
}

impl ShareGenerator for GpuSharing {
    fn generate(&mut self, secrets: &[Secret]) -> SdaClientResult<Vec<Vec<Share>>> {
        let n = self.scheme.output_size();
        let len = unsafe { sda_share_length(&self.c, secrets.len() as u64) } as usize;
        let draws = self.draws(secrets.len(), len);
        let mut flat = vec![0_i64; n * len];
        let c = self.c;
        self.dev.call(|h| unsafe {
            sda_share_generate(h, &c, secrets.as_ptr(), secrets.len() as u64, draws.as_ptr(), draws.len() as u64,
                               flat.as_mut_ptr(), flat.len() as u64)
        })?;
        // [clerk][batch], batched.rs:25-28
        Ok((0..n).map(|j| flat[j * len..(j + 1) * len].to_vec()).collect())
    }
}

impl ShareCombiner for GpuSharing {
    fn combine(&self, shares: &Vec<Vec<Share>>) -> SdaClientResult<Vec<Share>> {
        let (ptrs, lens) = rows_of(shares);
        let mut out = vec![0_i64; shares.get(0).map_or(0, |r| r.len())];
        let mut out_len = 0_u64;
        let c = self.c;
        self.dev.call(|h| unsafe {
            sda_share_combine(h, &c, ptrs.as_ptr(), lens.as_ptr(), shares.len() as u64, out.as_mut_ptr(),
                              out.len() as u64, &mut out_len)
        })?;
        out.truncate(out_len as usize);
        Ok(out)
    }
}

/// SecretReconstructor (the factory's `dimension` argument, sharing/mod.rs:76).
pub struct GpuReconstructor {
    dev: Arc<Device>,
    c: SdaSharingScheme,
    dimension: usize,
}

impl GpuReconstructor {
    pub fn new(dev: Arc<Device>, scheme: &LinearSecretSharingScheme, dimension: usize) -> GpuReconstructor {
        GpuReconstructor { dev: dev, c: sharing_c(scheme), dimension: dimension }
    }
}

impl SecretReconstructor for GpuReconstructor {
    fn reconstruct(&self, indexed_shares: &Vec<(usize, Vec<Share>)>) -> SdaClientResult<Vec<Secret>> {
        let idx: Vec<u64> = indexed_shares.iter().map(|&(i, _)| i as u64).collect();
        let ptrs: Vec<*const i64> = indexed_shares.iter().map(|&(_, ref r)| r.as_ptr()).collect();
        let lens: Vec<u64> = indexed_shares.iter().map(|&(_, ref r)| r.len() as u64).collect();
        let widest = lens.iter().cloned().max().unwrap_or(0) as usize;
        let mut out = vec![0_i64; std::cmp::max(self.dimension, widest)];
        let mut out_len = 0_u64;
        let (c, dim) = (self.c, self.dimension as u64);
        self.dev.call(|h| unsafe {
            sda_secret_reconstruct(h, &c, dim, idx.as_ptr(), ptrs.as_ptr(), lens.as_ptr(), ptrs.len() as u64,
                                   out.as_mut_ptr(), out.len() as u64, &mut out_len)
        })?;
        out.truncate(out_len as usize);
        Ok(out)
    }
}

// ---------------------------------------------------------------- masking

/// SecretMasker + MaskCombiner + SecretUnmasker for the three LinearMaskingScheme variants.  The masking
/// traits return plain values, so engine errors panic, as the reference's asserts do.
pub struct GpuMasker {
    dev: Arc<Device>,
    scheme: LinearMaskingScheme,
    c: SdaMaskingScheme,
    rng: OsRng,
}

impl GpuMasker {
    pub fn new(dev: Arc<Device>, scheme: &LinearMaskingScheme) -> GpuMasker {
        GpuMasker {
            dev: dev,
            scheme: scheme.clone(),
            c: masking_c(scheme),
            rng: OsRng::new().expect("Unable to get randomness source"),
        }
    }
}

impl SecretMasker for GpuMasker {
    fn mask(&mut self, secrets: &[Secret]) -> (Vec<Mask>, Vec<MaskedSecret>) {
        // the draws the reference makes: Full, one gen_range(0, m) per element (full.rs:25-27); ChaCha, the
        // ceil(bits / 32) seed words (chacha.rs:29-33)
        let (seed, full): (Vec<u32>, Vec<i64>) = match self.scheme {
            LinearMaskingScheme::None => (vec![], vec![]),
            LinearMaskingScheme::Full { modulus } => {
                let rng = &mut self.rng;
                (vec![], secrets.iter().map(|_| rng.gen_range(0_i64, modulus)).collect())
            }
            LinearMaskingScheme::ChaCha { seed_bitsize, .. } => {
                let rng = &mut self.rng;
                ((0..(seed_bitsize + 31) / 32).map(|_| rng.next_u32()).collect(), vec![])
            }
        };
        let mut mask = vec![0_i64; std::cmp::max(secrets.len(), seed.len())];
        let mut masked = vec![0_i64; secrets.len()];
        let mut mask_len = 0_u64;
        let c = self.c;
        let full_ptr = if full.is_empty() { std::ptr::null() } else { full.as_ptr() };
        self.dev
            .call(|h| unsafe {
                sda_secret_mask(h, &c, secrets.as_ptr(), secrets.len() as u64, seed.as_ptr(), seed.len() as u64,
                                full_ptr, mask.as_mut_ptr(), mask.len() as u64, &mut mask_len, masked.as_mut_ptr())
            })
            .expect("mask");
        mask.truncate(mask_len as usize);
        (mask, masked)
    }
}

impl MaskCombiner for GpuMasker {
    fn combine(&self, masks: &Vec<Vec<Mask>>) -> Vec<Mask> {
        let (ptrs, lens) = rows_of(masks);
        let mut out = vec![0_i64; std::cmp::max(self.c.dimension as usize, masks.get(0).map_or(0, |r| r.len()))];
        let mut out_len = 0_u64;
        let c = self.c;
        self.dev
            .call(|h| unsafe {
                sda_mask_combine(h, &c, ptrs.as_ptr(), lens.as_ptr(), masks.len() as u64, out.as_mut_ptr(),
                                 out.len() as u64, &mut out_len)
            })
            .expect("mask combine");
        out.truncate(out_len as usize);
        out
    }
}

impl SecretUnmasker for GpuMasker {
    fn unmask(&self, values: &(Vec<Mask>, Vec<MaskedSecret>)) -> Vec<Secret> {
        let mut out = vec![0_i64; values.1.len()];
        let mut out_len = 0_u64;
        let c = self.c;
        self.dev
            .call(|h| unsafe {
                sda_secret_unmask(h, &c, values.0.as_ptr(), values.0.len() as u64, values.1.as_ptr(),
                                  values.1.len() as u64, out.as_mut_ptr(), out.len() as u64, &mut out_len)
            })
            .expect("unmask");
        out.truncate(out_len as usize);
        out
    }
}
