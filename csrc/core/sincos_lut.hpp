// Sine/cosine look-up table used by the time-domain resampling.
//
// 65 samples of sin/cos(2*pi*i/64) with 2*pi truncated to 6.283185f, rounded
// to 6 decimals. These exact float values define the resampling numerics of the
// reference (erp_utilities.cpp:45-46, lookup :176-209); the nearest-neighbour
// index of every resampled sample depends on them bit-for-bit, so host and
// device share this one table.
#pragma once

namespace brp {

constexpr int kLutRes = 64;
constexpr int kLutSize = kLutRes + 1;
constexpr float kLutTwoPi = 6.283185f;
constexpr float kLutTwoPiInv = 1.0f / 6.283185f;
constexpr float kLutResF = 64.0f;
constexpr float kLutResFInv = 1.0f / 64.0f;

constexpr float kSinLut[kLutSize] = {
    0.000000f, 0.098017f, 0.195090f, 0.290285f, 0.382683f, 0.471397f, 0.555570f, 0.634393f,
    0.707107f, 0.773010f, 0.831470f, 0.881921f, 0.923880f, 0.956940f, 0.980785f, 0.995185f,
    1.000000f, 0.995185f, 0.980785f, 0.956940f, 0.923880f, 0.881921f, 0.831470f, 0.773010f,
    0.707107f, 0.634393f, 0.555570f, 0.471397f, 0.382683f, 0.290285f, 0.195091f, 0.098017f,
    0.000000f, -0.098017f, -0.195090f, -0.290284f, -0.382683f, -0.471397f, -0.555570f, -0.634393f,
    -0.707107f, -0.773010f, -0.831469f, -0.881921f, -0.923880f, -0.956940f, -0.980785f, -0.995185f,
    -1.000000f, -0.995185f, -0.980785f, -0.956940f, -0.923880f, -0.881921f, -0.831470f, -0.773011f,
    -0.707107f, -0.634394f, -0.555570f, -0.471397f, -0.382684f, -0.290285f, -0.195091f, -0.098017f,
    -0.000000f};

constexpr float kCosLut[kLutSize] = {
    1.000000f, 0.995185f, 0.980785f, 0.956940f, 0.923880f, 0.881921f, 0.831470f, 0.773010f,
    0.707107f, 0.634393f, 0.555570f, 0.471397f, 0.382683f, 0.290285f, 0.195090f, 0.098017f,
    0.000000f, -0.098017f, -0.195090f, -0.290285f, -0.382683f, -0.471397f, -0.555570f, -0.634393f,
    -0.707107f, -0.773010f, -0.831470f, -0.881921f, -0.923880f, -0.956940f, -0.980785f, -0.995185f,
    -1.000000f, -0.995185f, -0.980785f, -0.956940f, -0.923880f, -0.881921f, -0.831470f, -0.773011f,
    -0.707107f, -0.634393f, -0.555570f, -0.471397f, -0.382684f, -0.290285f, -0.195090f, -0.098017f,
    0.000000f, 0.098017f, 0.195090f, 0.290285f, 0.382683f, 0.471397f, 0.555570f, 0.634393f,
    0.707107f, 0.773010f, 0.831470f, 0.881921f, 0.923879f, 0.956940f, 0.980785f, 0.995185f,
    1.000000f};

}  // namespace brp
