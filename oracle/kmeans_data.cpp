// kmeans_data.cpp -- the kmeans_smi host's input generator.
//
// TEST INFRASTRUCTURE ONLY (see smi_oracle.c's header): used to build the
// parity fixtures, never by smi_amd/.
//
// Restates examples/host/kmeans_smi.cpp:96-147 with the same standard-library
// engine and distributions -- libstdc++, where std::default_random_engine is
// std::minstd_rand0 -- so the tests run on exactly the points and initial
// centroids the reference host generates for the same arguments.
#include <cstddef>
#include <random>
#include <type_traits>

static_assert(std::is_same<std::default_random_engine, std::minstd_rand0>::value,
              "libstdc++'s default_random_engine is minstd_rand0");

extern "C" {

// Rank 0's generation, kmeans_smi.cpp:99-147: cluster means
// (clusters x dims), the input (num_points x dims, point i around mean
// i % clusters) and the initial centroids (clusters x dims, copies of random
// input points).  Returns 0, or -1 if the reference would copy a centroid
// from one past the end of its input (uniform_int_distribution(0,
// num_points) is inclusive, :141-146).
int oracle_kmeans_reference_data(int num_points, int clusters, int dims, float *means, float *input,
                                 float *centroids) {
    std::default_random_engine rng(5);
    std::uniform_real_distribution<float> dist_means(-5, 5);
    for (int k = 0; k < clusters; ++k)
        for (int d = 0; d < dims; ++d) means[(size_t)k * dims + d] = dist_means(rng);
    std::normal_distribution<float> normal_dist;
    for (int i = 0; i < num_points; i++) {
        const int k = i % clusters;
        for (int d = 0; d < dims; ++d) input[(size_t)i * dims + d] = normal_dist(rng) + means[(size_t)k * dims + d];
    }
    std::uniform_int_distribution<size_t> index_dist(0, num_points);
    int rc = 0;
    for (int k = 0; k < clusters; ++k) {
        const size_t i = index_dist(rng);
        if (i >= (size_t)num_points) {
            rc = -1;
            continue;
        }
        for (int d = 0; d < dims; ++d) centroids[(size_t)k * dims + d] = input[i * dims + d];
    }
    return rc;
}

// The C++ standard's check value for minstd_rand0 ([rand.predef]): the
// 10000th invocation of a default-constructed engine yields 1043618065.
unsigned long oracle_minstd_rand0_10000(void) {
    std::minstd_rand0 e;
    e.discard(9999);
    return e();
}
}
