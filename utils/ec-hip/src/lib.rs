//! `ec-hip`: the CESS segment -> fragment Reed-Solomon codec on MI355X (gfx950), a thin Rust layer
//! over libcessec's C ABI (`include/cess_ec.h`).
//!
//! The API follows `reed-solomon-erasure` (`ReedSolomon::new(k, m)`, `encode`, `reconstruct`,
//! `reconstruct_data`, `verify`) so the uploader / miner tools that produce the chain's records
//! (`SegmentList { hash, fragment_list }`, c-pallets/file-bank/src/types.rs:13-16, submitted with
//! `upload_declaration`, c-pallets/file-bank/src/lib.rs:419-428) swap codecs without changing
//! their call sites. `Pipeline` streams whole files through the GPU (pinned multi-buffered copies,
//! encode, GPU SegmentList hashes); `deal_info` builds the SCALE bytes of the extrinsic argument.
#![allow(non_camel_case_types)]

use std::ffi::CStr;
use std::os::raw::{c_char, c_int, c_longlong, c_void};

#[repr(C)]
pub struct cec_codec {
    _p: [u8; 0],
}
#[repr(C)]
pub struct cec_pipeline {
    _p: [u8; 0],
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct cec_pipeline_opts {
    pub shard_len: usize,
    pub batch_segments: usize,
    pub depth: c_int,
    pub hash: c_int,
    pub window: c_int,
    pub max_segments: u64,
    /// host SHA-256 threads for hash = 2 (host) / 3 (hybrid); 0 = 16
    pub host_threads: c_int,
    /// hash = 3: batches at the end of the last source hashed wholly on the host (-1 = auto)
    pub tail_batches: c_int,
}

/// `cec_pipeline_opts.hash`: where the SegmentList hashes run.
pub const CEC_PIPE_HASH_NONE: c_int = 0;
pub const CEC_PIPE_HASH_GPU: c_int = 1;
pub const CEC_PIPE_HASH_HOST: c_int = 2;
pub const CEC_PIPE_HASH_HYBRID: c_int = 3;

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct cec_pipeline_stats {
    pub segments: u64,
    pub bytes_in: u64,
    pub seconds: f64,
    pub read_seconds: f64,
    pub wait_seconds: f64,
}

pub type cec_read_fn = extern "C" fn(user: *mut c_void, dst: *mut u8, cap: usize) -> c_longlong;
pub type cec_fragments_fn =
    extern "C" fn(user: *mut c_void, seg: u64, shards: *const *const u8, shard_len: usize) -> c_int;
pub type cec_record_fn =
    extern "C" fn(user: *mut c_void, seg: u64, seg_hex: *const u8, frag_hex: *const u8) -> c_int;
pub type cec_file_fragments_fn = extern "C" fn(user: *mut c_void, file: usize, seg: u64,
                                               shards: *const *const u8, shard_len: usize)
                                               -> c_int;
pub type cec_file_record_fn = extern "C" fn(user: *mut c_void, file: usize, seg: u64,
                                            seg_hex: *const u8, frag_hex: *const u8) -> c_int;
pub type cec_file_done_fn =
    extern "C" fn(user: *mut c_void, file: usize, stats: *const cec_pipeline_stats) -> c_int;

/// One source of `cec_pipeline_run_files`: its read callback, that callback's user pointer and
/// the source's size in bytes (0 = unknown).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct cec_source {
    pub read: cec_read_fn,
    pub user: *mut c_void,
    pub size: u64,
}

extern "C" {
    pub fn cec_strerror(code: c_int) -> *const c_char;
    pub fn cec_last_error() -> *const c_char;
    pub fn cec_create(k: c_int, m: c_int, device: c_int, out: *mut *mut cec_codec) -> c_int;
    pub fn cec_destroy(c: *mut cec_codec);
    pub fn cec_encode(c: *mut cec_codec, shards: *const *mut u8, shard_len: usize) -> c_int;
    pub fn cec_reconstruct(c: *mut cec_codec, shards: *const *mut u8, present: *const u8,
                           shard_len: usize, data_only: c_int) -> c_int;
    pub fn cec_verify(c: *mut cec_codec, shards: *const *mut u8, shard_len: usize,
                      ok: *mut c_int) -> c_int;
    pub fn cec_pipeline_create(c: *mut cec_codec, opts: *const cec_pipeline_opts,
                               out: *mut *mut cec_pipeline) -> c_int;
    pub fn cec_pipeline_destroy(p: *mut cec_pipeline);
    pub fn cec_pipeline_run(p: *mut cec_pipeline, read: cec_read_fn,
                            on_fragments: Option<cec_fragments_fn>,
                            on_record: Option<cec_record_fn>, user: *mut c_void,
                            stats: *mut cec_pipeline_stats) -> c_int;
    pub fn cec_pipeline_info(p: *const cec_pipeline, window: *mut c_int,
                             device_slots: *mut c_int, depth: *mut c_int) -> c_int;
    pub fn cec_pipeline_run_files(p: *mut cec_pipeline, sources: *const cec_source,
                                  nsources: usize, on_fragments: Option<cec_file_fragments_fn>,
                                  on_record: Option<cec_file_record_fn>,
                                  on_done: Option<cec_file_done_fn>, user: *mut c_void,
                                  stats: *mut cec_pipeline_stats) -> c_int;
    pub fn cec_sha256_host(bufs: *const *const u8, n: usize, len: usize, hex: *mut u8,
                           prefix_len: usize, prefix_hex: *mut u8, threads: c_int) -> c_int;
    pub fn cec_sha256_host_state(bufs: *const *const u8, n: usize, len: usize, hex: *mut u8,
                                 state_out: *mut u32, threads: c_int) -> c_int;
    pub fn cec_host_sha_set_form(form: c_int) -> c_int;
    pub fn cec_host_sha_form() -> c_int;
    pub fn cec_host_sha_pool_threads() -> c_int;
    pub fn cec_host_sha_probe(form: c_int, bytes_per_chain: usize, chains: c_int) -> f64;
    pub fn cec_scale_deal_info(seg_hex: *const u8, frag_hex: *const u8, nseg: usize,
                               nfrag: usize, out: *mut u8, out_cap: usize,
                               out_len: *mut usize) -> c_int;
}

/// The rest of `include/cess_ec.h`, declared one to one (HBM-resident batches, hash queue,
/// audit chunks, records, the multi-GPU degraded read). Device pointers are `*mut u8` /
/// `*const u8`; HIP streams are `*mut c_void` (null = the null stream).
pub mod sys {
    use super::{cec_codec, c_char, c_int, c_void};

    #[repr(C)]
    pub struct cec_hashq {
        _p: [u8; 0],
    }
    #[repr(C)]
    pub struct cec_dist {
        _p: [u8; 0],
    }
    #[repr(C)]
    #[derive(Clone, Copy, Debug, Default)]
    pub struct cec_dist_move {
        pub seg: u64,
        pub frag: i32,
        pub src: i32,
        pub dst: i32,
        pub kind: i32,
    }
    pub const CEC_DIST_ID_BYTES: usize = 128;
    pub const CEC_DIST_SURVIVOR: i32 = 0;
    pub const CEC_DIST_PARTIAL: i32 = 1;
    pub const CEC_DIST_OPT_EXCHANGE: c_int = 1;
    pub const CEC_DIST_OPT_GROUP_OPS: c_int = 3;
    pub type cec_locate_fn = extern "C" fn(user: *mut c_void, seg: u64, frag: c_int) -> *const u8;

    extern "C" {
        pub fn cec_version() -> *const c_char;
        pub fn cec_device_count() -> c_int;
        pub fn cec_codec_info(c: *const cec_codec, k: *mut c_int, m: *mut c_int,
                              device: *mut c_int) -> c_int;
        pub fn cec_matrix(c: *const cec_codec, out: *mut u8) -> c_int;
        pub fn cec_encode_batch(c: *mut cec_codec, d_data: *const u8, d_parity: *mut u8,
                                nseg: usize, shard_len: usize, stream: *mut c_void) -> c_int;
        pub fn cec_reconstruct_batch(c: *mut cec_codec, d_data: *mut u8, d_parity: *mut u8,
                                     nseg: usize, shard_len: usize, present: *const u8,
                                     per_segment: c_int, data_only: c_int,
                                     stream: *mut c_void) -> c_int;
        pub fn cec_reconstruct_partial_batch(c: *mut cec_codec, d_data: *mut u8,
                                             d_parity: *mut u8, nseg: usize, shard_len: usize,
                                             present: *const u8, held: *const u8,
                                             data_only: c_int, stream: *mut c_void) -> c_int;
        pub fn cec_verify_batch(c: *mut cec_codec, d_data: *const u8, d_parity: *const u8,
                                nseg: usize, shard_len: usize, d_ok: *mut u8,
                                stream: *mut c_void) -> c_int;
        pub fn cec_xor_batch(d_dst: *mut u8, d_src: *const u8, nsrc: usize, src_stride: usize,
                             len: usize, stream: *mut c_void) -> c_int;
        pub fn cec_sha256_batch(c: *mut cec_codec, d_data: *const u8, d_parity: *const u8,
                                nseg: usize, shard_len: usize, d_hex: *mut u8,
                                stream: *mut c_void) -> c_int;
        pub fn cec_sha256_hex(d_bufs: *const *const u8, n: usize, len: usize, hex: *mut u8,
                              stream: *mut c_void) -> c_int;
        pub fn cec_hashq_create(device: c_int, capacity: usize, stream: *mut c_void,
                                out: *mut *mut cec_hashq) -> c_int;
        pub fn cec_hashq_destroy(q: *mut cec_hashq);
        pub fn cec_hashq_add(q: *mut cec_hashq, d_base: *const u8, n: usize, per: usize,
                             outer_stride: usize, inner_stride: usize, len: usize,
                             d_hex: *mut u8, hex_outer: usize, ticket: *mut u64) -> c_int;
        pub fn cec_hashq_add_resume(q: *mut cec_hashq, d_base: *const u8, n: usize, per: usize,
                                    outer_stride: usize, inner_stride: usize, len: usize,
                                    start_len: usize, d_states: *const u32, d_hex: *mut u8,
                                    hex_outer: usize, ticket: *mut u64) -> c_int;
        pub fn cec_hashq_add_prefix(q: *mut cec_hashq, d_base: *const u8, n: usize, per: usize,
                                    outer_stride: usize, inner_stride: usize, len: usize,
                                    d_hex: *mut u8, hex_outer: usize, prefix_len: usize,
                                    d_prefix_hex: *mut u8, prefix_hex_outer: usize,
                                    ticket: *mut u64) -> c_int;
        pub fn cec_hashq_tick(q: *mut cec_hashq, max_blocks: u32) -> c_int;
        pub fn cec_hashq_finish(q: *mut cec_hashq) -> c_int;
        pub fn cec_hashq_status(q: *const cec_hashq, ticket: u64, done: *mut c_int,
                                live_chains: *mut usize, blocks_left: *mut u64) -> c_int;
        pub fn cec_hashq_set_option(q: *mut cec_hashq, option: c_int, value: c_int) -> c_int;
        pub fn cec_split_segment(seg: *const u8, seg_len: usize, k: c_int,
                                 shards: *const *mut u8, shard_len: usize) -> c_int;
        pub fn cec_challenge_indices(randoms: *const u64, nrand: usize, chunk_count: u32,
                                     need: u32, out: *mut u32, used: *mut usize) -> c_int;
        pub fn cec_audit_chunks(c: *mut cec_codec, d_data: *const u8, d_parity: *const u8,
                                nseg: usize, shard_len: usize, chunk_count: u32,
                                indices: *const u32, nidx: u32, d_chunks: *mut u8,
                                d_hex: *mut u8, stream: *mut c_void) -> c_int;
        pub fn cec_scale_compact(n: u32, out: *mut u8, out_cap: usize, out_len: *mut usize)
                                 -> c_int;
        pub fn cec_scale_upload_declaration(file_hash_hex: *const u8, seg_hex: *const u8,
                                            frag_hex: *const u8, nseg: usize, nfrag: usize,
                                            account: *const u8, file_name: *const u8,
                                            file_name_len: usize, bucket_name: *const u8,
                                            bucket_name_len: usize, out: *mut u8,
                                            out_cap: usize, out_len: *mut usize) -> c_int;
        pub fn cec_shard_id(hash_hex: *const u8, index: u32, out68: *mut u8) -> c_int;
        pub fn cec_hash_from_shard_id(shard_id68: *const u8, hash_hex_out: *mut u8) -> c_int;
        pub fn cec_scale_upload_filler(tee_worker: *const u8, block_num: *const u32,
                                       miners: *const u8, filler_hex: *const u8, n: usize,
                                       out: *mut u8, out_cap: usize, out_len: *mut usize)
                                       -> c_int;
        pub fn cec_scale_generate_restoral_order(file_hash_hex: *const u8,
                                                 fragment_hex: *const u8, out: *mut u8,
                                                 out_cap: usize, out_len: *mut usize) -> c_int;
        pub fn cec_scale_claim_restoral_order(fragment_hex: *const u8, out: *mut u8,
                                              out_cap: usize, out_len: *mut usize) -> c_int;
        pub fn cec_scale_claim_restoral_exist_order(miner: *const u8, file_hash_hex: *const u8,
                                                    fragment_hex: *const u8, out: *mut u8,
                                                    out_cap: usize, out_len: *mut usize)
                                                    -> c_int;
        pub fn cec_scale_restoral_order_complete(fragment_hex: *const u8, out: *mut u8,
                                                 out_cap: usize, out_len: *mut usize) -> c_int;
        pub fn cec_audit_random_subject(pallet_id: *const u8, seed: u32, out12: *mut u8)
                                        -> c_int;
        pub fn cec_audit_random_u64(randomness: *const u8, len: usize, out: *mut u64) -> c_int;
        pub fn cec_survivors(k: c_int, m: c_int, present: *const u8, survivors: *mut u8) -> c_int;
        pub fn cec_challenge_random_list(randomness: *const u8, nrand: usize, need: u32,
                                         out: *mut u8, used: *mut usize) -> c_int;
        pub fn cec_fill_synthetic(d_out: *mut u8, seg_bytes: usize, nseg: usize, seg0: u64,
                                  seed: u64, stream: *mut c_void) -> c_int;
        pub fn cec_set_option(c: *mut cec_codec, option: c_int, value: c_int) -> c_int;
        pub fn cec_get_stat(c: *const cec_codec, stat: c_int, value: *mut u64) -> c_int;
        pub fn cec_dist_unique_id(id: *mut u8) -> c_int;
        pub fn cec_dist_create(c: *mut cec_codec, id: *const u8, world: c_int, rank: c_int,
                               out: *mut *mut cec_dist) -> c_int;
        pub fn cec_dist_destroy(d: *mut cec_dist);
        pub fn cec_dist_plan(k: c_int, m: c_int, world: c_int, lost_seg: *const u64,
                             lost_frag: *const u8, nlost: usize, moves: *mut cec_dist_move,
                             moves_cap: usize, nmoves: *mut usize, decoder: *mut i32) -> c_int;
        pub fn cec_dist_plan_ex(k: c_int, m: c_int, world: c_int, exchange: c_int,
                                lost_seg: *const u64, lost_frag: *const u8, nlost: usize,
                                moves: *mut cec_dist_move, moves_cap: usize, nmoves: *mut usize,
                                decoder: *mut i32) -> c_int;
        pub fn cec_dist_set_option(d: *mut cec_dist, option: c_int, value: c_int) -> c_int;
        pub fn cec_dist_groups(d: *const cec_dist, groups: *mut u64) -> c_int;
        pub fn cec_dist_plan_groups(k: c_int, m: c_int, world: c_int, exchange: c_int,
                                    group_ops: c_int, lost_seg: *const u64, lost_frag: *const u8,
                                    nlost: usize, starts: *mut u64, starts_cap: usize,
                                    ngroups: *mut usize) -> c_int;
        pub fn cec_dist_degraded_read(d: *mut cec_dist, lost_seg: *const u64,
                                      lost_frag: *const u8, nlost: usize, shard_len: usize,
                                      locate: cec_locate_fn, user: *mut c_void,
                                      d_out: *const *mut u8, stream: *mut c_void,
                                      nrebuilt: *mut usize) -> c_int;
    }
}

/// One rank's share of the multi-GPU degraded read (libcessec's own RCCL group): fragment f of
/// segment s lives on rank (s + f) mod world (random_assign_miner's spread,
/// c-pallets/file-bank/src/functions.rs:187-283).
pub struct DistGroup<'c> {
    d: *mut sys::cec_dist,
    _codec: std::marker::PhantomData<&'c ReedSolomon>,
}

extern "C" fn locate_cb(user: *mut c_void, seg: u64, frag: c_int) -> *const u8 {
    let f = unsafe { &mut *(user as *mut &mut dyn FnMut(u64, usize) -> *const u8) };
    f(seg, frag as usize)
}

impl<'c> DistGroup<'c> {
    /// A fresh group id (on one rank; hand it to the others out of band).
    pub fn unique_id() -> Result<[u8; sys::CEC_DIST_ID_BYTES], Error> {
        let mut id = [0u8; sys::CEC_DIST_ID_BYTES];
        check(unsafe { sys::cec_dist_unique_id(id.as_mut_ptr()) })?;
        Ok(id)
    }

    /// Join as `rank` of `world` (collective over the ranks).
    pub fn join(codec: &'c ReedSolomon, id: &[u8; sys::CEC_DIST_ID_BYTES], world: i32,
                rank: i32) -> Result<Self, Error> {
        let mut d = std::ptr::null_mut();
        check(unsafe { sys::cec_dist_create(codec.c, id.as_ptr(), world, rank, &mut d) })?;
        Ok(DistGroup { d, _codec: std::marker::PhantomData })
    }

    /// Exchange of later degraded reads: 0 survivors, 1 partial products, 2 per segment
    /// whichever moves fewer fragments (the default of a new group; the same value on every
    /// rank).
    pub fn set_exchange(&mut self, exchange: i32) -> Result<(), Error> {
        check(unsafe { sys::cec_dist_set_option(self.d, sys::CEC_DIST_OPT_EXCHANGE, exchange) })
    }

    /// At most `ops` point-to-point transfers per rank in one RCCL group (default 1024; 0 = one
    /// group per round of 256 segments; the same value on every rank).
    pub fn set_group_ops(&mut self, ops: i32) -> Result<(), Error> {
        check(unsafe { sys::cec_dist_set_option(self.d, sys::CEC_DIST_OPT_GROUP_OPS, ops) })
    }

    /// Transfer groups this handle has issued so far.
    pub fn groups(&self) -> Result<u64, Error> {
        let mut g = 0u64;
        check(unsafe { sys::cec_dist_groups(self.d, &mut g) })?;
        Ok(g)
    }

    /// Rebuild the `lost` (segment, fragment) list, the same on every rank; `locate(seg, frag)`
    /// gives the device address of a fragment this rank holds (null if absent); `out[i]` receives
    /// lost entry i when this rank rebuilds it. Returns the number rebuilt here.
    pub fn degraded_read(&mut self, lost: &[(u64, u8)], shard_len: usize,
                         mut locate: impl FnMut(u64, usize) -> *const u8,
                         out: &[*mut u8]) -> Result<usize, Error> {
        let segs: Vec<u64> = lost.iter().map(|l| l.0).collect();
        let frags: Vec<u8> = lost.iter().map(|l| l.1).collect();
        let mut f: &mut dyn FnMut(u64, usize) -> *const u8 = &mut locate;
        let mut n = 0usize;
        check(unsafe {
            sys::cec_dist_degraded_read(self.d, segs.as_ptr(), frags.as_ptr(), lost.len(),
                                        shard_len, locate_cb,
                                        &mut f as *mut _ as *mut c_void,
                                        if out.is_empty() { std::ptr::null() } else { out.as_ptr() },
                                        std::ptr::null_mut(), &mut n)
        })?;
        Ok(n)
    }
}

impl Drop for DistGroup<'_> {
    fn drop(&mut self) {
        unsafe { sys::cec_dist_destroy(self.d) }
    }
}

pub const CEC_ETOOFEW: c_int = -2;
pub const CEC_ESHARDLEN: c_int = -3;
pub const CEC_ESEGCOUNT: c_int = -9;
pub const SEGMENT_COUNT: usize = 1000; // runtime/src/lib.rs:1026
pub const FRAGMENT_COUNT: usize = 3; // runtime/src/lib.rs:1027

/// A libcessec error: the C code and its message.
#[derive(Debug, Clone, PartialEq, Eq)]
pub struct Error {
    pub code: i32,
    pub message: String,
}

impl Error {
    fn from_code(code: c_int) -> Self {
        let msg = unsafe {
            let s = CStr::from_ptr(cec_strerror(code)).to_string_lossy().into_owned();
            let d = CStr::from_ptr(cec_last_error()).to_string_lossy().into_owned();
            if d.is_empty() { s } else { format!("{s} ({d})") }
        };
        Error { code, message: msg }
    }
}

impl std::fmt::Display for Error {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "libcessec error {}: {}", self.code, self.message)
    }
}

impl std::error::Error for Error {}

fn check(code: c_int) -> Result<(), Error> {
    if code == 0 { Ok(()) } else { Err(Error::from_code(code)) }
}

/// One codec bound to one GPU (`reed_solomon_erasure::ReedSolomon` shape).
pub struct ReedSolomon {
    c: *mut cec_codec,
    k: usize,
    m: usize,
}

unsafe impl Send for ReedSolomon {}

impl ReedSolomon {
    pub fn new(data_shards: usize, parity_shards: usize) -> Result<Self, Error> {
        Self::on_device(data_shards, parity_shards, 0)
    }

    pub fn on_device(data_shards: usize, parity_shards: usize, device: i32) -> Result<Self, Error> {
        let mut c = std::ptr::null_mut();
        check(unsafe { cec_create(data_shards as c_int, parity_shards as c_int, device, &mut c) })?;
        Ok(ReedSolomon { c, k: data_shards, m: parity_shards })
    }

    pub fn data_shard_count(&self) -> usize { self.k }
    pub fn parity_shard_count(&self) -> usize { self.m }
    pub fn total_shard_count(&self) -> usize { self.k + self.m }

    fn ptrs(shards: &mut [&mut [u8]]) -> Result<(Vec<*mut u8>, usize), Error> {
        let len = shards.first().map(|s| s.len()).unwrap_or(0);
        if len == 0 || shards.iter().any(|s| s.len() != len) {
            return Err(Error::from_code(CEC_ESHARDLEN));
        }
        Ok((shards.iter_mut().map(|s| s.as_mut_ptr()).collect(), len))
    }

    /// Parity shards `shards[k..]` from data shards `shards[..k]`, in place.
    pub fn encode(&self, shards: &mut [&mut [u8]]) -> Result<(), Error> {
        if shards.len() != self.k + self.m {
            return Err(Error::from_code(CEC_ETOOFEW));
        }
        let (p, len) = Self::ptrs(shards)?;
        check(unsafe { cec_encode(self.c, p.as_ptr(), len) })
    }

    pub fn verify(&self, shards: &mut [&mut [u8]]) -> Result<bool, Error> {
        let (p, len) = Self::ptrs(shards)?;
        let mut ok: c_int = 0;
        check(unsafe { cec_verify(self.c, p.as_ptr(), len, &mut ok) })?;
        Ok(ok != 0)
    }

    fn reconstruct_inner(&self, shards: &mut [Option<Vec<u8>>], data_only: bool) -> Result<(), Error> {
        let n = self.k + self.m;
        if shards.len() != n {
            return Err(Error::from_code(CEC_ETOOFEW));
        }
        let len = shards.iter().flatten().map(|s| s.len()).next().ok_or(Error::from_code(CEC_ETOOFEW))?;
        let present: Vec<u8> = shards.iter().map(|s| s.is_some() as u8).collect();
        for (i, s) in shards.iter_mut().enumerate() {
            if s.is_none() && (i < self.k || !data_only) {
                *s = Some(vec![0u8; len]);
            }
        }
        let mut scratch = vec![0u8; len];
        let p: Vec<*mut u8> = shards
            .iter_mut()
            .map(|s| match s { Some(v) => v.as_mut_ptr(), None => scratch.as_mut_ptr() })
            .collect();
        check(unsafe { cec_reconstruct(self.c, p.as_ptr(), present.as_ptr(), len, data_only as c_int) })
    }

    /// Recreate every missing (`None`) shard.
    pub fn reconstruct(&self, shards: &mut [Option<Vec<u8>>]) -> Result<(), Error> {
        self.reconstruct_inner(shards, false)
    }

    /// Recreate only the missing data shards.
    pub fn reconstruct_data(&self, shards: &mut [Option<Vec<u8>>]) -> Result<(), Error> {
        self.reconstruct_inner(shards, true)
    }
}

impl Drop for ReedSolomon {
    fn drop(&mut self) {
        unsafe { cec_destroy(self.c) }
    }
}

/// One segment's SegmentList hashes: 64 hex chars for the segment, k+m for its fragments.
#[derive(Clone, Debug, PartialEq, Eq)]
pub struct SegmentList {
    pub hash: [u8; 64],
    pub fragment_list: Vec<[u8; 64]>,
}

struct Ctx<'a, R: std::io::Read> {
    src: &'a mut R,
    n: usize,
    on_fragments: &'a mut dyn FnMut(u64, &[&[u8]]),
    records: Vec<SegmentList>,
    err: Option<std::io::Error>,
}

extern "C" fn read_cb<R: std::io::Read>(user: *mut c_void, dst: *mut u8, cap: usize) -> c_longlong {
    let ctx = unsafe { &mut *(user as *mut Ctx<R>) };
    let buf = unsafe { std::slice::from_raw_parts_mut(dst, cap) };
    match ctx.src.read(buf) {
        Ok(n) => n as c_longlong,
        Err(e) => {
            ctx.err = Some(e);
            -1
        }
    }
}

extern "C" fn frag_cb<R: std::io::Read>(user: *mut c_void, seg: u64, shards: *const *const u8,
                                        shard_len: usize) -> c_int {
    let ctx = unsafe { &mut *(user as *mut Ctx<R>) };
    let v: Vec<&[u8]> = (0..ctx.n)
        .map(|i| unsafe { std::slice::from_raw_parts(*shards.add(i), shard_len) })
        .collect();
    (ctx.on_fragments)(seg, &v);
    0
}

extern "C" fn rec_cb<R: std::io::Read>(user: *mut c_void, _seg: u64, seg_hex: *const u8,
                                       frag_hex: *const u8) -> c_int {
    let ctx = unsafe { &mut *(user as *mut Ctx<R>) };
    let mut hash = [0u8; 64];
    hash.copy_from_slice(unsafe { std::slice::from_raw_parts(seg_hex, 64) });
    let fh = unsafe { std::slice::from_raw_parts(frag_hex, 64 * ctx.n) };
    let fragment_list = fh.chunks(64).map(|c| { let mut h = [0u8; 64]; h.copy_from_slice(c); h }).collect();
    ctx.records.push(SegmentList { hash, fragment_list });
    0
}

/// libcessec's host pipeline (pinned multi-buffered H2D / encode / D2H, GPU hashes).
pub struct Pipeline<'c> {
    p: *mut cec_pipeline,
    n: usize,
    _codec: std::marker::PhantomData<&'c ReedSolomon>,
}

impl<'c> Pipeline<'c> {
    pub fn new(codec: &'c ReedSolomon, opts: cec_pipeline_opts) -> Result<Self, Error> {
        let mut p = std::ptr::null_mut();
        check(unsafe { cec_pipeline_create(codec.c, &opts, &mut p) })?;
        Ok(Pipeline { p, n: codec.k + codec.m, _codec: std::marker::PhantomData })
    }

    /// Stream a file through the GPU: `on_fragments(seg, shards)` sees each segment's k+m
    /// shards, the returned records are the file's SegmentLists in segment order.
    pub fn run<R: std::io::Read>(&mut self, src: &mut R,
                                 on_fragments: &mut dyn FnMut(u64, &[&[u8]]))
                                 -> Result<(Vec<SegmentList>, cec_pipeline_stats), Error> {
        let mut ctx = Ctx { src, n: self.n, on_fragments, records: Vec::new(), err: None };
        let mut st = cec_pipeline_stats::default();
        let rc = unsafe {
            cec_pipeline_run(self.p, read_cb::<R>, Some(frag_cb::<R>), Some(rec_cb::<R>),
                             &mut ctx as *mut Ctx<R> as *mut c_void, &mut st)
        };
        if let Some(e) = ctx.err.take() {
            return Err(Error { code: rc, message: e.to_string() });
        }
        check(rc)?;
        Ok((ctx.records, st))
    }
}

impl Drop for Pipeline<'_> {
    fn drop(&mut self) {
        unsafe { cec_pipeline_destroy(self.p) }
    }
}

/// SCALE bytes of `deal_info: BoundedVec<SegmentList, SegmentCount>` for upload_declaration.
pub fn deal_info(segments: &[SegmentList]) -> Result<Vec<u8>, Error> {
    let nfrag = segments.first().map(|s| s.fragment_list.len()).unwrap_or(FRAGMENT_COUNT);
    let seg: Vec<u8> = segments.iter().flat_map(|s| s.hash).collect();
    let frag: Vec<u8> = segments.iter().flat_map(|s| s.fragment_list.iter().flatten().copied()).collect();
    let mut len = 0usize;
    check(unsafe { cec_scale_deal_info(seg.as_ptr(), frag.as_ptr(), segments.len(), nfrag,
                                       std::ptr::null_mut(), 0, &mut len) })?;
    let mut out = vec![0u8; len];
    check(unsafe { cec_scale_deal_info(seg.as_ptr(), frag.as_ptr(), segments.len(), nfrag,
                                       out.as_mut_ptr(), len, &mut len) })?;
    Ok(out)
}

/// Size-query-then-fill of a libcessec SCALE encoder (`f(out, cap, &mut len)`).
fn scale_call(f: impl Fn(*mut u8, usize, *mut usize) -> c_int) -> Result<Vec<u8>, Error> {
    let mut len = 0usize;
    check(f(std::ptr::null_mut(), 0, &mut len))?;
    let mut out = vec![0u8; len];
    check(f(out.as_mut_ptr(), len, &mut len))?;
    Ok(out)
}

/// `FillerInfo` of c-pallets/file-bank/src/types.rs:82-86.
#[derive(Clone, Debug)]
pub struct FillerInfo {
    pub block_num: u32,
    pub miner_address: [u8; 32],
    pub filler_hash: [u8; 64],
}

/// Call data of `upload_filler(tee_worker, filler_list)` (call 8, at most 10 fillers).
pub fn upload_filler(tee_worker: &[u8; 32], fillers: &[FillerInfo]) -> Result<Vec<u8>, Error> {
    let blk: Vec<u32> = fillers.iter().map(|f| f.block_num).collect();
    let miners: Vec<u8> = fillers.iter().flat_map(|f| f.miner_address).collect();
    let hex: Vec<u8> = fillers.iter().flat_map(|f| f.filler_hash).collect();
    scale_call(|o, c, l| unsafe {
        sys::cec_scale_upload_filler(tee_worker.as_ptr(), blk.as_ptr(), miners.as_ptr(),
                                     hex.as_ptr(), fillers.len(), o, c, l)
    })
}

/// Call data of `restoral_order_complete(fragment_hash)` (call 16): emit it only after the
/// rebuilt fragment's SHA-256 hex equals `fragment_hash`.
pub fn restoral_order_complete(fragment_hash: &[u8; 64]) -> Result<Vec<u8>, Error> {
    scale_call(|o, c, l| unsafe { sys::cec_scale_restoral_order_complete(fragment_hash.as_ptr(), o, c, l) })
}

/// Call data of `claim_restoral_order(restoral_fragment)` (call 14).
pub fn claim_restoral_order(fragment_hash: &[u8; 64]) -> Result<Vec<u8>, Error> {
    scale_call(|o, c, l| unsafe { sys::cec_scale_claim_restoral_order(fragment_hash.as_ptr(), o, c, l) })
}
