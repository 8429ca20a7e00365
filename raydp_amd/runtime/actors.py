"""Actor manager (filled in by the actor-runtime milestone)."""


class ActorManager:
    def __init__(self, node):
        self.node = node

    def on_node_removed(self, node_id):
        pass

    def shutdown(self):
        pass
