/* C restatement of GravitySim's KDK loop — TEST ORACLE / CPU BASELINE ONLY.
 *
 * Follows datasets/nbody/dataset/synthetic_sim.py:
 *   compute_acceleration  318-340  a_i = G * sum_j m_j (x_j - x_i) (|x_j - x_i|^2 + eps^2)^-1.5
 *   simulate_step         342-355  v += a dt/2 ; x += v dt ; a = A(x) ; v += a dt/2
 *   sample_trajectory     383-408  sample (pos, vel, acc*mass) every sample_freq steps, BEFORE stepping
 * Per system, single thread, j summed in ascending order like the reference's
 * (dx*inv_r3) @ mass.  Built by oracle/Makefile into oracle/_build/.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static void accel(int N, const double* pos, const double* mass, double G, double soft2, double* acc) {
    for (int i = 0; i < N; ++i) {
        double ax = 0.0, ay = 0.0, az = 0.0;
        for (int j = 0; j < N; ++j) {
            double dx = pos[3 * j + 0] - pos[3 * i + 0];
            double dy = pos[3 * j + 1] - pos[3 * i + 1];
            double dz = pos[3 * j + 2] - pos[3 * i + 2];
            double r2 = dx * dx + dy * dy + dz * dz + soft2;
            double inv = r2 > 0.0 ? pow(r2, -1.5) : r2;
            ax += dx * inv * mass[j];
            ay += dy * inv * mass[j];
            az += dz * inv * mass[j];
        }
        acc[3 * i + 0] = G * ax;
        acc[3 * i + 1] = G * ay;
        acc[3 * i + 2] = G * az;
    }
}

/* pos/vel [S,N,3] (updated in place to the final state), mass [S,N];
 * saves [S, T/freq, N, 3].  Returns 0, or -1 on bad arguments. */
int oracle_gravity_sample(int64_t S, int64_t N, int64_t T, int64_t freq, double dt, double G, double soft,
                          double* pos, double* vel, const double* mass,
                          double* pos_save, double* vel_save, double* force_save) {
    if (S < 0 || N <= 0 || T < 0 || freq <= 0 || T % freq) return -1;
    const int64_t Ts = T / freq;
    double* acc = (double*)malloc(sizeof(double) * 3 * N);
    if (!acc) return -1;
    for (int64_t s = 0; s < S; ++s) {
        double* p = pos + s * N * 3;
        double* v = vel + s * N * 3;
        const double* m = mass + s * N;
        accel((int)N, p, m, G, soft * soft, acc);
        int64_t c = 0;
        for (int64_t t = 0; t < T; ++t) {
            if (t % freq == 0) {
                double* ps = pos_save + (s * Ts + c) * N * 3;
                double* vs = vel_save + (s * Ts + c) * N * 3;
                double* fs = force_save + (s * Ts + c) * N * 3;
                memcpy(ps, p, sizeof(double) * 3 * N);
                memcpy(vs, v, sizeof(double) * 3 * N);
                for (int64_t i = 0; i < N; ++i)
                    for (int k = 0; k < 3; ++k) fs[3 * i + k] = acc[3 * i + k] * m[i];
                ++c;
            }
            for (int64_t i = 0; i < 3 * N; ++i) v[i] += acc[i] * dt / 2.0;
            for (int64_t i = 0; i < 3 * N; ++i) p[i] += v[i] * dt;
            accel((int)N, p, m, G, soft * soft, acc);
            for (int64_t i = 0; i < 3 * N; ++i) v[i] += acc[i] * dt / 2.0;
        }
    }
    free(acc);
    return 0;
}
