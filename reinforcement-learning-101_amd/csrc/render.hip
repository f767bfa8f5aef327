// render.hip — dd_render: the rgb_array frame of DroneGame.render
// (reference delivery_drone/game/game_engine.py:300-337) for a batch of lanes.
//
// The reference draws with pygame: sky fill, ground rect (:312-315),
// Platform.render (platform.py:76-102), Drone.render + _render_thrust
// (drone.py:155-218), _render_hud (game_engine.py:339-384) and, once the
// game is over, _render_game_over (:386-412); rgb_array mode returns
// surfarray.array3d(screen).transpose(1, 0, 2), i.e. [H][W][3] uint8.  Here a
// frame is one pass of a per-pixel kernel that evaluates the same scene in
// painter's order for 4 consecutive pixels per lane (12 output bytes), one
// grid row per rendered lane, so the lane's state is wave-uniform (scalar
// loads) and the frame leaves as contiguous stores: the kernel is bound by
// the bytes it writes (1.44 MB per 800 x 600 frame).
//
// pygame is not installed here, so these are restatements of its primitive
// rules, not pixel-verified against it ("Rendering"):
//   * rect (l, t, w, h): pixels l <= X < l + w, t <= Y < t + h; an outline of
//     width 2 is the rect's pixels within 2 of an edge;
//   * a vertical line of width 2 from (cx, t) to (cx, b): columns cx, cx + 1,
//     rows t..b inclusive;
//   * filled circle (c, r): (X - cx)^2 + (Y - cy)^2 <= r^2; filled ellipse in
//     rect (l, t, w, h): pixel centres inside the inscribed ellipse;
//   * transform.rotate(surface, -angle) + blit centred on (x, y): every pixel
//     centre is rotated back into the 40 x 20 drone sprite and takes the
//     sprite pixel it lands on (nearest neighbour), transparent outside;
//   * text: pygame.font.Font(None, 24 | 30 | 48) is stood in for by DejaVu
//     Sans Bold at 16 / 20 / 33 px (font_atlas.h); anti-aliased glyph
//     coverage a blends as pygame's ALPHA_BLEND: d += ((s - d) * a + s) >> 8;
//   * the game-over overlay (surface alpha 128, black): d += (-d * 128) >> 8.
// Geometry of the rotated parts is computed in float32 from float32-rounded
// sin / cos of the angle, so the CPU restatement (oracle/render.py) gets the
// same pixels; numbers in the HUD are formatted like Python's f-strings
// (correctly rounded, ties to even).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dronestep.h"
#include "font_atlas.h"
#include "trig.h"

namespace dd {
namespace render {

constexpr int kBlock = 256;
constexpr int kPix = 4;    // consecutive pixels per lane and pass (12 output bytes)
constexpr int kQuads = 8;  // passes per lane: a block covers kBlock * kPix * kQuads = 8,192 pixels
constexpr int kTexts = 10;
constexpr int kMaxChars = 32;
constexpr double kDeg2Rad = 3.14159265358979323846 / 180.0;

// colours, 0x00BBGGRR (config.py:9-15 and the literals of the render code)
__host__ __device__ constexpr uint32_t rgb(uint32_t r, uint32_t g, uint32_t b) { return r | (g << 8) | (b << 16); }
constexpr uint32_t kSky = rgb(135, 206, 235), kGround = rgb(101, 67, 33), kPlatform = rgb(50, 205, 50),
                   kOutline = rgb(0, 150, 0), kWhite = rgb(255, 255, 255), kDrone = rgb(200, 200, 200),
                   kRotor = rgb(100, 100, 100), kHub = rgb(50, 50, 50), kThrust = rgb(255, 100, 0),
                   kBarBg = rgb(50, 50, 50), kGreen = rgb(0, 255, 0), kYellow = rgb(255, 255, 0),
                   kRed = rgb(255, 0, 0);
constexpr int kDroneW = 40;  // config.DRONE_WIDTH (the sprite; the physics never reads it)

// One string of the frame, laid out: its chars, the glyph and left edge of
// each, and (built per block) the char under every column of its box.
constexpr int kMaxTextW = 640;
// The fixed text of each string (index 10: the title of a crash).
__device__ constexpr char kPrefix[11][20] = {"Fuel: ", "Speed: ", "Angle: ", "Distance: ", "Episode: ",
                                             "Steps: ", "H", "SUCCESSFUL LANDING!", "Total Reward: ",
                                             "Press R to restart", "CRASHED!"};

struct Text {
    int32_t x0, y0, w, h, face, len;
    uint32_t color;
    uint8_t s[kMaxChars];
    int16_t glyph[kMaxChars];
    int16_t start[kMaxChars];
    int32_t r0, roff;  // this block's first row of it, and where those rows sit in the raster (-1: not staged)
};

// Per block, the coverage of the rows of each drawn string that fall in the
// block's rows, staged in LDS once, so a text pixel is one LDS read: read
// straight from the atlas in global memory, a HUD block waited on a chain of
// dependent loads per pass (strings x pixels x passes).
constexpr int kRaster = 16384;
// Rows of a string the raster fill loads at once per column: all that one block's pixels touch when the
// image is 800 wide (8,192 consecutive pixels: at most 12 rows); narrower images take several rounds.
constexpr int kBlockRows = 12;

// ---- f-string formatting (Python's int() / str(int) / format(x, '.Nf')) ----
struct Str {
    uint8_t* c;
    int n;
    __device__ void put(char ch) {
        if (n < kMaxChars) c[n++] = (uint8_t)ch;
    }
    __device__ void put(const char* lit) {
        while (*lit) put(*lit++);
    }
    __device__ void put_u64(uint64_t v) {
        char tmp[20];
        int k = 0;
        while (v >> 32) { tmp[k++] = (char)('0' + v % 10); v /= 10; }  // 64-bit division only above 2^32
        uint32_t w = (uint32_t)v;
        do { tmp[k++] = (char)('0' + w % 10u); w /= 10u; } while (w);
        while (k) put(tmp[--k]);
    }
    // format(x, '.1f') / '.0f': the correctly rounded decimal, ties to even,
    // "-" for a set sign bit (Python prints -0.0 as "-0.0").  x * 10 is split
    // into its rounded product p and the exact remainder e = fma(x, 10, -p),
    // so a tie of p is resolved by the sign of e.  |x| >= 2^50 prints the
    // integer part only (never reached by a frame's values).
    __device__ void put_fixed(double x, int decimals) {
        if (__builtin_isnan(x)) { put("nan"); return; }
        if (__builtin_signbit(x)) put('-');
        x = fabs(x);
        if (__builtin_isinf(x)) { put("inf"); return; }
        if (x >= 1125899906842624.0) { put_u64((uint64_t)x); return; }
        const double scale = decimals ? 10.0 : 1.0;
        const double p = x * scale;
        const double e = fma(x, scale, -p);
        double r = rint(p);
        const double d = p - r;
        if (d == 0.5 && e > 0.0) r += 1.0;
        else if (d == -0.5 && e < 0.0) r -= 1.0;
        const uint64_t q = (uint64_t)r;
        if (decimals) { put_u64(q / 10); put('.'); put((char)('0' + q % 10)); } else { put_u64(q); }
    }
};

// pygame's per-pixel-alpha blit: d += ((s - d) * a + s) >> 8, per channel
__device__ __forceinline__ uint32_t blend(uint32_t d, uint32_t s, int a) {
    uint32_t out = 0;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const int dc = (int)((d >> (8 * ch)) & 255u), sc = (int)((s >> (8 * ch)) & 255u);
        out |= (uint32_t)(dc + (((sc - dc) * a + sc) >> 8)) << (8 * ch);
    }
    return out;
}

// the game-over overlay, black at surface alpha 128: d + ((-d * 128) >> 8)
// = d - ceil(d / 2) = floor(d / 2) per channel, i.e. every byte halved
__device__ __forceinline__ uint32_t darken(uint32_t d) { return (d >> 1) & 0x7F7F7Fu; }

// The font tables a block reads while laying out and drawing its strings,
// copied to LDS once (the layout walks them char by char: from global
// memory that was a chain of dependent loads per string).
struct FontLds {
    int16_t index[font::kFaces * 128];
    uint8_t advance[font::kGlyphs];
    uint32_t offset[font::kGlyphs];
};

// string t blended over colour d at pixel (X, Y) (pygame ALPHA_BLEND of the
// glyph's coverage); d unchanged outside its box
__device__ __forceinline__ uint32_t draw_text(uint32_t d, const Text& t, const uint8_t* cc, const FontLds& fl,
                                              const uint8_t* raster, int X, int Y) {
    const int u = X - t.x0, v = Y - t.y0;
    if (u < 0 || u >= t.w || v < 0 || v >= t.h || t.len == 0) return d;
    int a;
    if (t.roff >= 0) {
        a = raster[t.roff + (Y - t.r0) * t.w + u];
    } else {  // did not fit the raster: from the atlas
        const int i = cc[u];
        const int g = t.glyph[i];
        a = font::kAtlas[fl.offset[g] + v * fl.advance[g] + (u - t.start[i])];
    }
    return a ? blend(d, t.color, a) : d;
}

// the strings of `mask` over a lane's 4 pixels (X0 .. X0 + 3, row Y), each
// only where its rows and columns meet them
__device__ __forceinline__ void draw_texts(uint32_t (&px4)[kPix], uint32_t mask, const Text* texts,
                                           const uint8_t (*colchar)[kMaxTextW], const FontLds& fl,
                                           const uint8_t* raster, int X0, int Y) {
    for (uint32_t m = mask; m; m &= m - 1) {
        const int k = __builtin_ctz(m);
        const Text& t = texts[k];
        if (Y < t.y0 || Y >= t.y0 + t.h || X0 + kPix <= t.x0 || X0 >= t.x0 + t.w) continue;
#pragma unroll
        for (int j = 0; j < kPix; ++j) px4[j] = draw_text(px4[j], t, colchar[k], fl, raster, X0 + j, Y);
    }
}

struct Args {
    const uint8_t* actions;  // [N] bitmask of the last step (nullable: no flames)
    const int32_t* lanes;    // [count] lanes to draw (nullable: 0..count-1)
    uint8_t* rgb;            // [count][H][W][3]
    int32_t width, height, ground, count;
    int64_t n;               // lanes in the SoA
    int32_t phw, phh, dhh;   // platform half width / height, drone half height (px)
    int32_t flags;
};

template <typename T>
struct View {
    const T *x, *y, *vx, *vy, *angle, *fuel, *px, *py, *total;
    const uint8_t* status;
    const int32_t *steps, *episode;
};

template <typename T>
__global__ __launch_bounds__(kBlock) void render_kernel(Args p, View<T> v) {
    __shared__ Text texts[kTexts];
    __shared__ uint8_t colchar[kTexts][kMaxTextW];
    __shared__ uint8_t raster[kRaster];
    __shared__ FontLds fl;
    const int slot = blockIdx.y;
    const int lane = p.lanes ? p.lanes[slot] : slot;
    if (lane < 0 || lane >= p.n) {  // not a lane: an all-zero frame
        for (int q = 0; q < kQuads; ++q) {
            const int t = (blockIdx.x * kQuads + q) * kBlock + threadIdx.x;
            if (t * kPix < p.width * p.height) {
                uint32_t* dst = reinterpret_cast<uint32_t*>(p.rgb + ((size_t)slot * p.width * p.height + (size_t)t * kPix) * 3);
                __builtin_nontemporal_store(0u, dst);
                __builtin_nontemporal_store(0u, dst + 1);
                __builtin_nontemporal_store(0u, dst + 2);
            }
        }
        return;
    }
    // the lane's state: wave-uniform
    const double x = (double)v.x[lane], y = (double)v.y[lane], angle = (double)v.angle[lane];
    const double fuel = (double)v.fuel[lane], px = (double)v.px[lane], py = (double)v.py[lane];
    const uint32_t status = v.status[lane];
    // flames: the last step's thrusters; none on a fresh episode (Drone.reset clears them)
    const uint32_t act = (p.actions && v.steps[lane] > 0) ? (p.actions[lane] & 7u) : 0u;
    const int W = p.width, H = p.height;
    const int first = blockIdx.x * kBlock * kPix * kQuads;  // this block's first pixel
    const int row_lo = first / W, row_hi = min(H - 1, (first + kBlock * kPix * kQuads - 1) / W);

    // float32 geometry of the rotated parts (see the header)
    double sd, cd;
    trig::sincos(angle * kDeg2Rad, &sd, &cd);
    const float s = (float)sd, c = (float)cd;
    const float xf = (float)x, yf = (float)y;
    const float hw = 0.5f * kDroneW, hh = (float)p.dhh;
    // _render_thrust flame centres: rotate_point(...) then int(x + fx), int(y + fy)
    const bool lit = fuel > 0.0;
    const bool main_on = (act & 1u) && lit, left_on = (act & 2u) && lit, right_on = (act & 4u) && lit;
    const float flame = hh + 15.0f / 2.0f;  // height / 2 + flame_length / 2
    const int mx = (int)(xf + (0.0f * c - flame * s)), my = (int)(yf + (0.0f * s + flame * c));
    const float sl = hw + 10.0f / 2.0f;  // width / 2 + side_flame_length / 2
    const int lx = (int)(xf + (-sl * c - 0.0f * s)), ly = (int)(yf + (-sl * s + 0.0f * c));
    const int rx = (int)(xf + (sl * c - 0.0f * s)), ry = (int)(yf + (sl * s + 0.0f * c));
    // platform bounds (platform.py:51-62), pygame truncating the float rect
    const int pl = (int)(px - p.phw), pt = (int)(py - p.phh), pw = 2 * p.phw, ph = 2 * p.phh;
    const int pcx = (int)px, pby = (int)(py + p.phh);
    const bool hud = p.flags & DD_RENDER_HUD;
    const bool over = (p.flags & DD_RENDER_GAME_OVER) && (status & DD_ST_DONE);

    // Block culling: a block covers 8,192 consecutive pixels (11-12 rows),
    // so each group of primitives is tested against the block's rows once
    // (a scalar branch) and most blocks only fill sky or ground.
    //   pad band: the platform and its centre line (pt .. bottom);
    //   drone band: the sprite (radius 22.4) and the flames (<= 30 px out);
    //   strings: only those whose rows meet the block's are laid out.
    const bool blk_pad = row_hi >= pt && row_lo <= pby;
    const bool blk_drone = (float)row_hi + 48.0f >= yf && (float)row_lo - 48.0f <= yf;
    // string k: where (y0 follows from the face height alone) and whether it is drawn
    int tx[kTexts], ty[kTexts], tface[kTexts];
    bool ton[kTexts], tcentre[kTexts];
    {
        const int hud_y[6] = {12, 40, 65, 90, 10, 35};
        const int hud_x[6] = {15, 10, 10, 10, W - 150, W - 150};
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            tx[k] = hud_x[k]; ty[k] = hud_y[k]; tface[k] = 0; ton[k] = hud; tcentre[k] = false;
        }
        tx[6] = pcx; ty[6] = (int)py; tface[6] = 1; ton[6] = true; tcentre[6] = true;  // the pad's "H"
        const int over_y[3] = {H / 2 - 30, H / 2 + 20, H / 2 + 50};
#pragma unroll
        for (int k = 7; k < kTexts; ++k) {
            tx[k] = W / 2; ty[k] = over_y[k - 7]; tface[k] = k == 7 ? 2 : 0; ton[k] = over; tcentre[k] = true;
        }
    }
    uint32_t need = 0;  // strings this block draws (wave-uniform)
#pragma unroll
    for (int k = 0; k < kTexts; ++k) {
        const int h = font::kHeight[tface[k]];
        const int y0 = tcentre[k] ? ty[k] - h / 2 : ty[k];
        if (ton[k] && row_hi >= y0 && row_lo < y0 + h) need |= 1u << k;
    }
    if (need) {
        for (int i = threadIdx.x; i < font::kFaces * 128; i += kBlock) fl.index[i] = font::kIndex[i];
        for (int i = threadIdx.x; i < font::kGlyphs; i += kBlock) {
            fl.advance[i] = font::kAdvance[i];
            fl.offset[i] = font::kOffset[i];
        }
        __syncthreads();
        const int k = threadIdx.x;
        if (k < kTexts && ((need >> k) & 1u)) {
            Text& t = texts[k];
            Str str{t.s, 0};
            // One code path for all ten strings (they are laid out by ten lanes
            // of one wave): prefix from a table, then at most one number.
            //   0 f"Fuel: {int(fuel)}"      (15, 12)   5 f"Steps: {steps}"     (W - 150, 35)
            //   1 f"Speed: {speed:.1f}"     (10, 40)   6 "H", centred on the pad
            //   2 f"Angle: {angle:.1f}°"    (10, 65)   7 game-over title, (W // 2, H // 2 - 30)
            //   3 f"Distance: {dist:.0f}"   (10, 90)   8 f"Total Reward: {total:.1f}" (W // 2, H // 2 + 20)
            //   4 f"Episode: {episode}"     (W - 150, 10)  9 "Press R to restart" (W // 2, H // 2 + 50)
            const double vx = (double)v.vx[lane], vy = (double)v.vy[lane], dx = px - x, dy = py - y;
            const bool landed = (status & DD_ST_LANDED) != 0;
            const int pre = k == 7 ? (landed ? 7 : 10) : k;
            double num = 0.0;
            int decimals = -1;  // -1: no number; 0: integer or .0f; 1: .1f
            switch (k) {  // selects only: every lane runs the same instructions
                case 0: num = (double)(int64_t)fuel; decimals = 0; break;
                case 1: num = sqrt(vx * vx + vy * vy); decimals = 1; break;
                case 2: num = angle; decimals = 1; break;
                case 3: num = sqrt(dx * dx + dy * dy); decimals = 0; break;
                case 4: num = (double)v.episode[lane]; decimals = 0; break;
                case 5: num = (double)v.steps[lane]; decimals = 0; break;
                case 8: num = (double)v.total[lane]; decimals = 1; break;
                default: break;
            }
            for (const char* c = kPrefix[pre]; *c; ++c) str.put(*c);
            if (decimals >= 0) str.put_fixed(num, decimals);
            if (k == 2) str.put((char)font::kDegree);
            const uint32_t color = k != 7 ? kWhite : landed ? kGreen : kRed;
            const int face = tface[k];
            int w = 0, n = 0;
            for (int i = 0; i < str.n; ++i) {  // glyphs with a cell in this face, side by side
                const int g = fl.index[face * 128 + (t.s[i] & 127)];
                if (g < 0) continue;
                t.glyph[n] = (int16_t)g;
                t.start[n] = (int16_t)w;
                w += fl.advance[g];
                ++n;
            }
            t.len = n;
            t.face = face;
            t.color = color;
            t.h = font::kHeight[face];
            t.w = min(w, kMaxTextW);
            // get_rect(center=...): x = cx - w // 2, y = cy - h // 2
            t.x0 = tcentre[k] ? tx[k] - w / 2 : tx[k];
            t.y0 = tcentre[k] ? ty[k] - t.h / 2 : ty[k];
        }
        __syncthreads();
        if (threadIdx.x == 0) {  // raster slots for the block's rows of each string
            int off = 0;
            for (uint32_t m = need; m; m &= m - 1) {
                Text& t = texts[__builtin_ctz(m)];
                t.r0 = max(t.y0, row_lo);
                const int bytes = max(0, min(t.y0 + t.h, row_hi + 1) - t.r0) * t.w;
                t.roff = off + bytes <= kRaster ? off : -1;
                if (t.roff >= 0) off += bytes;
            }
        }
        // the char under every column of each string drawn here
        for (uint32_t m = need; m; m &= m - 1) {
            const int k2 = __builtin_ctz(m);
            const Text& t = texts[k2];
            for (int u = threadIdx.x; u < t.w; u += kBlock) {
                int i = 0;
                while (i + 1 < t.len && t.start[i + 1] <= u) ++i;
                colchar[k2][u] = (uint8_t)i;
            }
        }
        __syncthreads();
        for (uint32_t m = need; m; m &= m - 1) {  // stage the coverage: independent loads, all lanes
            const int k2 = __builtin_ctz(m);
            const Text& t = texts[k2];
            if (t.roff < 0 || t.w == 0) continue;
            const int rows = max(0, min(t.y0 + t.h, row_hi + 1) - t.r0);
            for (int u = threadIdx.x; u < t.w; u += kBlock) {  // a column per lane: its rows loaded together
                const int i = colchar[k2][u];
                const int adv = fl.advance[t.glyph[i]];
                const uint8_t* src = font::kAtlas + fl.offset[t.glyph[i]] + (t.r0 - t.y0) * adv + (u - t.start[i]);
                for (int rb = 0; rb < rows; rb += kBlockRows) {
                    uint8_t col[kBlockRows];
#pragma unroll
                    for (int r = 0; r < kBlockRows; ++r) col[r] = rb + r < rows ? src[(rb + r) * adv] : 0;
#pragma unroll
                    for (int r = 0; r < kBlockRows; ++r)
                        if (rb + r < rows) raster[t.roff + (rb + r) * t.w + u] = col[r];
                }
            }
        }
        __syncthreads();
    }

    const bool blk_bar = hud && row_lo < 30;  // the fuel bar's rows
    const int fuel_w = (int)(200.0 * (fuel / 1000.0));  // fuel_bar_width * fuel_percent
    const double fpct = fuel / 1000.0;
    const uint32_t fuel_color = fpct > 0.3 ? kGreen : fpct > 0.1 ? kYellow : kRed;
    for (int q = 0; q < kQuads; ++q) {  // pass q: the block's q-th run of kBlock * kPix pixels
        const int t0 = (blockIdx.x * kQuads + q) * kBlock + threadIdx.x;
        if (t0 * kPix >= W * H) break;
        const int Y = (t0 * kPix) / W, X0 = (t0 * kPix) - Y * W;
        // Each primitive is gated by the pass's row first (the lane's 4 pixels
        // share Y, and a wave's 256 pixels span one or two rows), so a pass
        // through sky or ground costs a handful of instructions.
        const uint32_t base = Y >= p.ground ? kGround : kSky;
        uint32_t px4[kPix] = {base, base, base, base};
        if (blk_pad && Y >= pt && Y <= pby) {  // Platform.render: fill, 2-px outline, centre line
#pragma unroll
            for (int j = 0; j < kPix; ++j) {
                const int X = X0 + j;
                if (X >= pl && X < pl + pw && Y < pt + ph) {
                    const bool edge = X < pl + 2 || X >= pl + pw - 2 || Y < pt + 2 || Y >= pt + ph - 2;
                    px4[j] = edge ? kOutline : kPlatform;
                }
                if (X == pcx || X == pcx + 1) px4[j] = kWhite;
            }
        }
        draw_texts(px4, need & 0x40u, texts, colchar, fl, raster, X0, Y);  // the pad's "H"
        if (blk_drone && fabsf(((float)Y + 0.5f) - yf) <= hw + hh + 1.0f) {
#pragma unroll
            for (int j = 0; j < kPix; ++j) {
                const int X = X0 + j;
                // Drone.render: the sprite rotated about (x, y), nearest neighbour
                const float dx = ((float)X + 0.5f) - xf, dy = ((float)Y + 0.5f) - yf;
                if (fabsf(dx) <= hw + hh + 1.0f) {
                    const float u = dx * c + dy * s, w = dy * c - dx * s;
                    const float su = floorf(u + hw), sv = floorf(w + hh);
                    if (su >= 0.0f && su < (float)kDroneW && sv >= 0.0f && sv < 2.0f * hh) {
                        const int i = (int)su, k = (int)sv, cy = (int)hh;  // rotor / hub centres at height // 2
                        const int d0 = (i - kDroneW / 2) * (i - kDroneW / 2) + (k - cy) * (k - cy);
                        const int d1 = (i - 5) * (i - 5) + (k - cy) * (k - cy);
                        const int d2 = (i - (kDroneW - 5)) * (i - (kDroneW - 5)) + (k - cy) * (k - cy);
                        px4[j] = d0 <= 9 ? kHub : (d1 <= 25 || d2 <= 25) ? kRotor : kDrone;
                    }
                }
                // _render_thrust: main flame ellipse (fx - 8, fy - 7, 16, 15), side circles r = 5
                if (main_on) {
                    const float ex = ((float)X + 0.5f - (float)mx) / 8.0f;
                    const float ey = ((float)Y + 0.5f - ((float)(my - 7) + 7.5f)) / 7.5f;
                    if (ex * ex + ey * ey <= 1.0f) px4[j] = kThrust;
                }
                if (left_on && (X - lx) * (X - lx) + (Y - ly) * (Y - ly) <= 25) px4[j] = kThrust;
                if (right_on && (X - rx) * (X - rx) + (Y - ry) * (Y - ry) <= 25) px4[j] = kThrust;
            }
        }
        // _render_hud
        if (blk_bar && Y >= 10 && Y < 30) {
#pragma unroll
            for (int j = 0; j < kPix; ++j) {
                const int X = X0 + j;
                if (X >= 10 && X < 210) px4[j] = X < 10 + fuel_w ? fuel_color : kBarBg;
            }
        }
        draw_texts(px4, need & 0x3Fu, texts, colchar, fl, raster, X0, Y);
        // _render_game_over
        if (over) {
#pragma unroll
            for (int j = 0; j < kPix; ++j) px4[j] = darken(px4[j]);
            draw_texts(px4, need & 0x380u, texts, colchar, fl, raster, X0, Y);
        }
        // 4 RGB pixels = 3 dwords, little-endian byte order R G B R G B ...
        const uint32_t w0 = (px4[0] & 0xFFFFFFu) | (px4[1] << 24);
        const uint32_t w1 = ((px4[1] >> 8) & 0xFFFFu) | (px4[2] << 16);
        const uint32_t w2 = ((px4[2] >> 16) & 0xFFu) | (px4[3] << 8);
        uint32_t* dst = reinterpret_cast<uint32_t*>(p.rgb + ((size_t)slot * W * H + (size_t)t0 * kPix) * 3);
        __builtin_nontemporal_store(w0, dst);
        __builtin_nontemporal_store(w1, dst + 1);
        __builtin_nontemporal_store(w2, dst + 2);
    }
}

template <typename T>
View<T> view_of(const DDState& st) {
    View<T> v;
    v.x = (const T*)st.x; v.y = (const T*)st.y; v.vx = (const T*)st.vx; v.vy = (const T*)st.vy;
    v.angle = (const T*)st.angle; v.fuel = (const T*)st.fuel; v.px = (const T*)st.px; v.py = (const T*)st.py;
    v.total = (const T*)st.total_reward;
    v.status = st.status; v.steps = st.steps; v.episode = st.episode;
    return v;
}

// an integer-valued double in [lo, hi]
inline bool whole(double d, double lo, double hi) { return d >= lo && d <= hi && d == (double)(int64_t)d; }

}  // namespace render
}  // namespace dd

extern "C" int dd_render(const DDConfig* cfg, const DDState* st, const uint8_t* actions, const int32_t* lanes,
                         int64_t count, int64_t n, uint8_t* rgb, int32_t flags, void* stream) {
    using namespace dd::render;
    if (!cfg || !st || count < 0 || n < 0 || (!lanes && count > n)) return (int)hipErrorInvalidValue;
    if (count == 0) return 0;
    if (!rgb || !st->x || !st->y || !st->vx || !st->vy || !st->angle || !st->fuel || !st->px || !st->py ||
        !st->total_reward || !st->status || !st->steps || !st->episode)
        return (int)hipErrorInvalidValue;
    if (!whole(cfg->world_width, 4, 16384) || !whole(cfg->world_height, 1, 16384) ||
        ((int64_t)cfg->world_width % 4) != 0 || !whole(cfg->ground_level, -1e6, 1e6) ||
        !whole(cfg->platform_half_width, 0, 4096) || !whole(cfg->platform_half_height, 0, 4096) ||
        !whole(cfg->drone_half_height, 1, 64) || count > 65535)
        return (int)hipErrorInvalidValue;
    Args p;
    p.actions = actions;
    p.lanes = lanes;
    p.rgb = rgb;
    p.width = (int32_t)cfg->world_width;
    p.height = (int32_t)cfg->world_height;
    p.ground = (int32_t)cfg->ground_level;
    p.count = (int32_t)count;
    p.n = n;
    p.phw = (int32_t)cfg->platform_half_width;
    p.phh = (int32_t)cfg->platform_half_height;
    p.dhh = (int32_t)cfg->drone_half_height;
    p.flags = flags;
    const int64_t quads = ((int64_t)p.width * p.height / kPix + kQuads - 1) / kQuads;
    dim3 grid((unsigned)((quads + kBlock - 1) / kBlock), (unsigned)count);
    hipStream_t s = (hipStream_t)stream;
    if (st->precision == DD_F64)
        render_kernel<double><<<grid, kBlock, 0, s>>>(p, view_of<double>(*st));
    else if (st->precision == DD_F32)
        render_kernel<float><<<grid, kBlock, 0, s>>>(p, view_of<float>(*st));
    else
        return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
}
