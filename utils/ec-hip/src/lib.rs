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
}

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
    pub fn cec_scale_deal_info(seg_hex: *const u8, frag_hex: *const u8, nseg: usize,
                               nfrag: usize, out: *mut u8, out_cap: usize,
                               out_len: *mut usize) -> c_int;
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
