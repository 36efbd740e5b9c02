// GeePs facade (include/geeps.hpp) over the MI355X ClientLib.
// Same forwarding as the reference's src/client/geeps.cpp:41-132, including the
// num_val_limit = rows * ROW_DATA_SIZE passed for every batch op.
#include "geeps.hpp"

#include <cstdlib>

#include "check.hpp"
#include "client.hpp"

using geeps::ClientLib;
using geeps::OpInfo;
using geeps::client_lib;

namespace {

OpInfo make_op(OpInfo::Type type) {
  OpInfo op;
  op.type = type;
  return op;
}

// Apps may exit without Shutdown() (apps/helloworld does): let queued server
// work and device copies finish before the HIP runtime is torn down.
void quiesce_at_exit() {
  if (client_lib) client_lib->quiesce();
}

ClientLib &lib() {
  GP_CHECK_MSG(client_lib, "GeePs used before construction or after Shutdown");
  return *client_lib;
}

}  // namespace

GeePs::GeePs(uint process_id, const GeePsConfig &config) {
  GP_CHECK_MSG(!client_lib, "only one GeePs instance per process (as in the reference)");
  client_lib = new ClientLib(process_id, config);
  static bool registered = false;
  if (!registered) {
    std::atexit(quiesce_at_exit);
    registered = true;
  }
}

void GeePs::Shutdown() {
  if (!client_lib) return;
  client_lib->shutdown();
  delete client_lib;
  client_lib = nullptr;
}

std::string GeePs::GetStats() { return lib().json_stats(); }

void GeePs::StartIterations() { lib().start_iterations(); }

int GeePs::VirtualRead(size_t table_id, const vector<size_t> &row_ids, int slack) {
  OpInfo op = make_op(OpInfo::READ);
  op.table = table_id;
  op.rows = row_ids;
  op.slack = slack;
  op.num_vals_limit = row_ids.size() * ROW_DATA_SIZE;
  return lib().virtual_op(std::move(op));
}

int GeePs::VirtualPostRead(int prestep_handle) {
  OpInfo op = make_op(OpInfo::POST_READ);
  op.prestep_handle = prestep_handle;
  return lib().virtual_op(std::move(op));
}

int GeePs::VirtualPreUpdate(size_t table_id, const vector<size_t> &row_ids) {
  OpInfo op = make_op(OpInfo::PRE_WRITE);
  op.table = table_id;
  op.rows = row_ids;
  op.num_vals_limit = row_ids.size() * ROW_DATA_SIZE;
  return lib().virtual_op(std::move(op));
}

int GeePs::VirtualUpdate(int prestep_handle) {
  OpInfo op = make_op(OpInfo::WRITE);
  op.prestep_handle = prestep_handle;
  return lib().virtual_op(std::move(op));
}

int GeePs::VirtualLocalAccess(const vector<size_t> &row_ids, bool fetch) {
  OpInfo op = make_op(OpInfo::READ);
  op.table = 0xdeadbeef;  // table id is irrelevant for local access (geeps.cpp:76-82)
  op.rows = row_ids;
  op.num_vals_limit = row_ids.size() * ROW_DATA_SIZE;
  op.local = true;
  op.fetch = fetch;
  return lib().virtual_op(std::move(op));
}

int GeePs::VirtualPostLocalAccess(int prestep_handle, bool keep) {
  OpInfo op = make_op(OpInfo::POST_READ);
  op.prestep_handle = prestep_handle;
  op.local = true;
  op.keep = keep;
  return lib().virtual_op(std::move(op));
}

int GeePs::VirtualClock() { return lib().virtual_op(make_op(OpInfo::CLOCK)); }

void GeePs::FinishVirtualIteration() { lib().finish_virtual_iteration(); }

bool GeePs::Read(int handle, RowData **buffer_ptr) { return lib().read_batch(buffer_ptr, handle); }

void GeePs::PostRead(int handle) { lib().postread_batch(handle); }

void GeePs::PreUpdate(int handle, RowOpVal **buffer_ptr) {
  lib().preupdate_batch(buffer_ptr, handle);
}

void GeePs::Update(int handle) { lib().update_batch(handle); }

bool GeePs::LocalAccess(int handle, RowData **buffer_ptr) {
  return lib().read_batch(buffer_ptr, handle);
}

void GeePs::PostLocalAccess(int handle) { lib().postread_batch(handle); }

void GeePs::Clock() { lib().iterate(); }
