// rt_common.hpp — shared host-side helpers of the C ABI (error slot, small vector math).
#pragma once

#include <cmath>
#include <cstdint>
#include <string>

#include "rt_mi355x.h"

namespace rt {

// Per-thread last-error message behind rt_last_error(); set_error returns the code so
// call sites can `return set_error(RT_ERR_ARG, "...")`.
int set_error(int code, const std::string& msg);
void clear_error();

// Knob id's value set through rt_tuning_set, else dflt (include/rt_mi355x.h, rt_tune_id).
double tuning(int id, double dflt);

// Float vector helpers with the reference's evaluation order (G/include/vec3.h:327-348).
inline rt_vec3 v3(float x, float y, float z) { return rt_vec3{x, y, z}; }
inline rt_vec3 operator+(rt_vec3 a, rt_vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline rt_vec3 operator-(rt_vec3 a, rt_vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline rt_vec3 operator*(rt_vec3 a, float t) { return v3(a.x * t, a.y * t, a.z * t); }
inline rt_vec3 operator*(rt_vec3 a, rt_vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
// Vec3 / double: the double quotient rounded to float (vec3.h:334).
inline rt_vec3 div_d(rt_vec3 a, double t) {
    return v3(float(double(a.x) / t), float(double(a.y) / t), float(double(a.z) / t));
}
// Vec3 / Vec3 elementwise float division (vec3.h:333).
inline rt_vec3 div_v(rt_vec3 a, rt_vec3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
inline float dot(rt_vec3 u, rt_vec3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
inline rt_vec3 cross(rt_vec3 u, rt_vec3 v) {
    return v3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}

}  // namespace rt
