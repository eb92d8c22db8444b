// ip_common.h -- device helpers shared by the two hole-fill files
// (ofd_inpaint.hip: layered Telea; ofd_inpaint_seq.hip: cv2's sequential
// order).  Internal to the library; included inside an anonymous namespace.
#pragma once

constexpr float T_FAR = 1.0e6f;  // cv2's initial distance; an INSIDE pixel reads as this

// numpy float32 -> uint8 on x86 (utils.py:148): truncate through int32, keep the low byte
__device__ __forceinline__ unsigned to_u8(float v) {
    if (!(v > -2147483648.0f && v < 2147483648.0f)) return 0u;
    return unsigned(int(v)) & 0xFFu;
}

// cv::saturate_cast<uchar>(float): round half to even, clamp
__device__ __forceinline__ unsigned sat_u8(float v) {
    const float r = __builtin_rintf(v);
    return r < 0.f ? 0u : (r > 255.f ? 255u : unsigned(r));
}

// FastMarching_solve (double), with cv2's flag cases
__device__ __forceinline__ float fm_solve(float t1, bool in1, float t2, bool in2) {
    const double a11 = t1, a22 = t2;
    const double m12 = a11 < a22 ? a11 : a22;
    double sol;
    if (!in1) {
        if (!in2) {
            if (fabs(a11 - a22) >= 1.0)
                sol = 1 + m12;
            else
                sol = (a11 + a22 + sqrt(double(2 - (a11 - a22) * (a11 - a22)))) * 0.5;
        } else {
            sol = 1 + a11;
        }
    } else if (!in2) {
        sol = 1 + a22;
    } else {
        sol = 1 + m12;
    }
    return float(sol);
}

__device__ __forceinline__ float min4f(float a, float b, float c, float d) {
    const float x = a < b ? a : b, y = c < d ? c : d;
    return x < y ? x : y;
}
