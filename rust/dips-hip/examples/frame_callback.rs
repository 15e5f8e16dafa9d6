//! The reference's per-frame pattern through the binding: one
//! `frame_callback` (dips/src/lib.rs:233-246) per decoded RGBA8 frame, as the
//! GStreamer appsink closure drives it (dips/src/frame_extractor.rs:232-240),
//! then the difference series of the same clip.
//!
//!     cargo run --release --example frame_callback -- 3840 2160 64
use dips_hip::{frame_callback, ChromaFilter, ComputeState, DiPsFilter, DiffSeries, Mode, PixelFormat};
use std::time::Instant;

fn main() -> Result<(), Box<dyn std::error::Error>> {
    let args: Vec<u32> = std::env::args().skip(1).map(|a| a.parse().unwrap()).collect();
    let (w, h, n) = (*args.first().unwrap_or(&1920), *args.get(1).unwrap_or(&1080), *args.get(2).unwrap_or(&32));
    let fb = (w * h * 4) as usize;
    // a synthetic clip: a bright square moving over a gradient
    let clip: Vec<u8> = (0..n as usize * fb)
        .map(|i| {
            let (t, p) = (i / fb, (i % fb) / 4);
            let (x, y) = ((p % w as usize) as u32, (p / w as usize) as u32);
            let inside = x.wrapping_sub(8 * t as u32) < 64 && y < 64;
            if i % 4 == 3 { 255 } else if inside { 250 } else { ((x + y) & 0xFF) as u8 }
        })
        .collect();

    let mut cs = ComputeState::new(false, 1, 5.0, DiPsFilter::Unfiltered, ChromaFilter::None)?;
    let t = Instant::now();
    let mut last = Vec::new();
    for f in clip.chunks_exact(fb) {
        last = frame_callback(w, h, f, &mut cs);
    }
    let dt = t.elapsed().as_secs_f64();
    println!("{n} frame_callback calls at {w}x{h}: {:.1} frames/s (last output {} bytes)", n as f64 / dt, last.len());

    // the north-star series of the same frames, RGBA8, against the previous frame
    let mut ds = DiffSeries::new(PixelFormat::Rgba8, Mode::PerFrame, 8.0 / 255.0, ChromaFilter::None, 0)?;
    let series = ds.run(w, h, &clip, None, None)?;
    for (t, e) in series.iter().enumerate().take(4) {
        println!("frame {t}: sad {} sj {} count {} si {:.6}", e.sad, e.sj, e.count, dips_hip::series_si(e));
    }
    Ok(())
}
