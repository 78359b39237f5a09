// Drop-in for the reference istft.h (istft.h:6-42): same class and function. The tables are
// computed on the host exactly as istft.cpp:7-32 does; istft() runs the fused gfx950 iSTFT
// kernel (csrc/hip/istft.hip) on the process's default MI355X (MIO_DEVICE, else LOCAL_RANK,
// else 0) with host buffers in and out, as the reference's signature requires.
#pragma once

#include <memory>
#include <vector>

// Precomputed iSTFT cache (Hann window + IRFFT trig tables).
class istft_cache {
public:
    istft_cache(int n_fft, int win_length);
    ~istft_cache();

    int n_fft() const;
    int win_length() const;
    int n_freq() const;
    int n_mid() const;
    const std::vector<float> & cos_table() const;
    const std::vector<float> & sin_table() const;
    const std::vector<float> & nyquist_sign() const;
    const std::vector<float> & hann_window() const;

    struct gpu_state;                       // device + kernel handle, created on first use
    gpu_state * gpu(int device = -1) const;

private:
    int n_fft_ = 0;
    int win_length_ = 0;
    int n_freq_ = 0;
    int n_mid_ = 0;

    std::vector<float> cos_table_;    // [n_fft, n_mid]
    std::vector<float> sin_table_;    // [n_fft, n_mid]
    std::vector<float> nyquist_sign_; // [n_fft]
    std::vector<float> hann_window_;  // [win_length]

    mutable std::unique_ptr<gpu_state> gpu_;
};

// Inverse STFT via IRFFT + overlap-add (spec layout and output length as istft.h:32-42).
std::vector<float> istft(
    const float * spec,
    int n_frames,
    int hop_length,
    const istft_cache & cache);
