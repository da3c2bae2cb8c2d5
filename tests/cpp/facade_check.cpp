// Compile-and-run check of include/uvio_hp.hpp (the C++ facade) on a host without a GPU: the options load
// through the facade, Manager construction fails loudly with UVIO_HP_E_DEVICE (no CPU fallback), and every
// facade method is instantiated (taking their addresses forces the templates and inline bodies to compile).
#include <cstdio>
#include <cstring>

#include "uvio_hp.hpp"

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  uvio_hp_options_t o;
  if (uvio_hp_options_default(&o) != 0 || uvio_hp_options_load(argv[1], &o) != 0) return 3;
  auto f1 = &uvio_amd::Manager::msckf_update;
  auto f2 = &uvio_amd::Manager::slam_update;
  auto f3 = &uvio_amd::Manager::slam_delayed_init;
  auto f4 = &uvio_amd::Manager::feed_measurement_camera;
  auto f5 = &uvio_amd::Manager::feed_measurement_simulation;
  auto f6 = &uvio_amd::Manager::uwb_update_single;
  auto f7 = &uvio_amd::Manager::set_state;
  auto f8 = &uvio_amd::Manager::covariance;
  auto f9 = &uvio_amd::Manager::state_vector;
  auto f10 = &uvio_amd::Manager::propagate_and_clone;
  (void)f1, (void)f2, (void)f3, (void)f4, (void)f5, (void)f6, (void)f7, (void)f8, (void)f9, (void)f10;
  try {
    uvio_amd::Manager m(argv[1], 0);
    std::printf("created\n");
    return 4;
  } catch (const uvio_amd::Error &e) {
    std::printf("code %d: %s\n", e.code, e.what());
    return e.code == UVIO_HP_E_DEVICE ? 0 : 5;
  }
}
