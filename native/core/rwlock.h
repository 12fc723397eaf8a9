// Writer-preferring reader/writer lock for the scheduler ledger.
//
// std::shared_mutex on glibc is a reader-preferring pthread rwlock: while
// filter / prioritize sweeps (readers, one per extender call) overlap, a bind
// or release (writer) waits for a moment with NO reader, which under load
// never comes — measured: core bind waited 70-145 ms for the ledger at 1,250
// nodes.  Here a waiting writer stops new readers; readers never re-enter
// the lock recursively (a nested read behind a waiting writer would
// deadlock), which the ledger code already guarantees: only public entry
// points lock.
#pragma once
#include <pthread.h>

#include <system_error>

namespace kgwe {

class RwLock {
 public:
  RwLock() {
    pthread_rwlockattr_t a;
    pthread_rwlockattr_init(&a);
    pthread_rwlockattr_setkind_np(&a, PTHREAD_RWLOCK_PREFER_WRITER_NONRECURSIVE_NP);
    pthread_rwlock_init(&l_, &a);
    pthread_rwlockattr_destroy(&a);
  }
  ~RwLock() { pthread_rwlock_destroy(&l_); }
  RwLock(const RwLock&) = delete;
  RwLock& operator=(const RwLock&) = delete;

  void lock() { check(pthread_rwlock_wrlock(&l_)); }
  bool try_lock() { return pthread_rwlock_trywrlock(&l_) == 0; }
  void unlock() { pthread_rwlock_unlock(&l_); }
  void lock_shared() { check(pthread_rwlock_rdlock(&l_)); }
  bool try_lock_shared() { return pthread_rwlock_tryrdlock(&l_) == 0; }
  void unlock_shared() { pthread_rwlock_unlock(&l_); }

 private:
  static void check(int rc) {
    if (rc) throw std::system_error(rc, std::generic_category(), "rwlock");
  }
  pthread_rwlock_t l_;
};

}  // namespace kgwe
