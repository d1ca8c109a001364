"""Trial status strings and job states (the reference's values, so stored
documents are interchangeable: hyperopt/base.py:55-79)."""

STATUS_NEW = 'new'
STATUS_RUNNING = 'running'
STATUS_SUSPENDED = 'suspended'
STATUS_OK = 'ok'
STATUS_FAIL = 'fail'
STATUS_STRINGS = (STATUS_NEW, STATUS_RUNNING, STATUS_SUSPENDED, STATUS_OK, STATUS_FAIL)

JOB_STATE_NEW, JOB_STATE_RUNNING, JOB_STATE_DONE, JOB_STATE_ERROR = range(4)
JOB_STATES = [JOB_STATE_NEW, JOB_STATE_RUNNING, JOB_STATE_DONE, JOB_STATE_ERROR]

# keys every stored trial document carries (base.py:81-90)
TRIAL_KEYS = ['tid', 'spec', 'result', 'misc', 'state', 'owner', 'book_time', 'refresh_time',
              'exp_key']
TRIAL_MISC_KEYS = ['tid', 'cmd', 'idxs', 'vals']
