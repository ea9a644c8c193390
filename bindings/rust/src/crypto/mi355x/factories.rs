//! The hooks the six reference factories call first (client/src/crypto/sharing/mod.rs:35-96,
//! client/src/crypto/masking/mod.rs:33-94).  Each returns Some(GPU trait object) when the CryptoModule
//! holds a device, else None and the factory goes on with its reference body, unchanged.
//! README.md shows the one line each factory gets.  UNCOMPILED (no cargo in this environment).

use super::{Device, GpuMasker, GpuReconstructor, GpuSharing};
use crypto::*;
use std::sync::Arc;

pub fn share_generator(gpu: &Option<Arc<Device>>, scheme: &LinearSecretSharingScheme) -> Option<Box<ShareGenerator>> {
    gpu.as_ref().map(|d| Box::new(GpuSharing::new(d.clone(), scheme)) as Box<ShareGenerator>)
}

pub fn share_combiner(gpu: &Option<Arc<Device>>, scheme: &LinearSecretSharingScheme) -> Option<Box<ShareCombiner>> {
    gpu.as_ref().map(|d| Box::new(GpuSharing::new(d.clone(), scheme)) as Box<ShareCombiner>)
}

pub fn secret_reconstructor(gpu: &Option<Arc<Device>>, scheme: &LinearSecretSharingScheme, dimension: usize)
                            -> Option<Box<SecretReconstructor>> {
    gpu.as_ref().map(|d| Box::new(GpuReconstructor::new(d.clone(), scheme, dimension)) as Box<SecretReconstructor>)
}

pub fn secret_masker(gpu: &Option<Arc<Device>>, scheme: &LinearMaskingScheme) -> Option<Box<SecretMasker>> {
    gpu.as_ref().map(|d| Box::new(GpuMasker::new(d.clone(), scheme)) as Box<SecretMasker>)
}

pub fn mask_combiner(gpu: &Option<Arc<Device>>, scheme: &LinearMaskingScheme) -> Option<Box<MaskCombiner>> {
    gpu.as_ref().map(|d| Box::new(GpuMasker::new(d.clone(), scheme)) as Box<MaskCombiner>)
}

pub fn secret_unmasker(gpu: &Option<Arc<Device>>, scheme: &LinearMaskingScheme) -> Option<Box<SecretUnmasker>> {
    gpu.as_ref().map(|d| Box::new(GpuMasker::new(d.clone(), scheme)) as Box<SecretUnmasker>)
}
