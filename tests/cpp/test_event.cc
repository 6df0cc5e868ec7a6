// tests/cpp/test_event.cc -- KingDB's Event (thread/event_manager.h:17-56) under
// the interleaving that hangs Database::Close: StorageEngine::Close calls
// flush_buffer.NotifyWait() (storage/storage_engine.h:110-111) while the data
// thread is still busy in the last flush's index update, and only THEN does
// the data thread reach flush_buffer.Wait() (storage_engine.h:262-311).  The
// reference's NotifyWait is a bare notify_one (:44-46): the notification is
// lost and Wait sleeps forever.  The hook build's patched Event
// (oracle/kingdb_hook.py) records it under the lock, so Wait returns.
//
// Built twice (tests/test_event_fix.py): against the patched header and
// against the reference's.  Prints "returned" (exit 0) or "lost wake-up"
// (exit 2, the waiter left sleeping) -- deterministic: a barrier makes the
// notification come before the waiter's Wait().
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <thread>
#include <unistd.h>

#include "util/order.h"
#include "thread/event_manager.h"

int main() {
  kdb::Event<std::vector<kdb::Order>> flush_buffer;
  std::mutex m;
  std::condition_variable cv;
  bool notified = false;
  std::atomic<bool> returned(false);
  std::thread data_thread([&] {
    {  // "the last flush's index update": hold here until Close has notified
      std::unique_lock<std::mutex> l(m);
      cv.wait(l, [&] { return notified; });
    }
    flush_buffer.Wait();   // the loop's next Wait (storage_engine.h:265)
    returned = true;
  });
  flush_buffer.NotifyWait();   // Close's notification, while the data thread is busy
  {
    std::lock_guard<std::mutex> l(m);
    notified = true;
  }
  cv.notify_one();
  for (int i = 0; i < 300 && !returned; i++) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  if (!returned) {
    printf("lost wake-up\n");
    fflush(stdout);
    _exit(2);   // the waiter sleeps forever; leave without joining it
  }
  data_thread.join();
  printf("returned\n");
  return 0;
}
